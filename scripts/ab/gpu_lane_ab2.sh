# Same-box A/B: lanes 2 / 3 / 4 in the driver-like short run (5 warm-up plies, 20 timed) and in steady state.
set -u
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
for W in "5 20" "24 40"; do
  set -- $W
  for L in 2 3 4 3 2; do
    timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline --lanes $L > gpurun_out/ab2/w$1_l$L.json 2> gpurun_out/ab2/err.txt
    rc=$?; echo "warmup $1 lanes $L rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab2/w$1_l$L.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab2/err.txt; exit $rc; fi
  done
done
