# Full -m gpu suite on the current build, then a lanes 2 / 3 A/B with the co-resident heads.
set -u
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fin/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fin/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/fin/gpu_tests.log | head -20; exit $rc; fi
for W in "5 20" "24 40"; do
  set -- $W
  for L in 2 3 2 3; do
    timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --lanes $L --no-cpu-baseline > gpurun_out/fin/b.json 2>gpurun_out/fin/err.txt || { tail -3 gpurun_out/fin/err.txt; exit 1; }
    echo "bench w$1 lanes $L: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/fin/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
  done
done
