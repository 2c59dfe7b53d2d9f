# Same-box A/B: packed tiles (default with two lanes) vs round-aligned tiles (--no-pack), short and steady.
set -u
mkdir -p gpurun_out/pk
export TMPDIR=/tmp
for W in "5 20" "24 40"; do
  set -- $W
  for X in "" "--no-pack" "" "--no-pack"; do
    timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline $X > gpurun_out/pk/b.json 2> gpurun_out/pk/err.txt || { tail -3 gpurun_out/pk/err.txt; exit 1; }
    echo "warmup $1 ${X:-pack}: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pk/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
  done
done
