# Batch leaf dedup: exactness tests, then same-box bench A/B (--no-leaf-dedup) in the driver's short
# form and in steady state.
set -u
mkdir -p gpurun_out/dd
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "dedup or invariants or full_size" --timeout 200 --timeout-method thread > gpurun_out/dd/tests.log 2>&1
rc=$?; tail -1 gpurun_out/dd/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/dd/tests.log | head -20; exit $rc; fi
for W in "5 20" "24 40"; do
  set -- $W
  for D in off on off on; do
    F=""; if [ $D = off ]; then F="--no-leaf-dedup"; fi
    timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline $F > gpurun_out/dd/b.json 2>gpurun_out/dd/err.txt || { tail -3 gpurun_out/dd/err.txt; exit 1; }
    echo "bench w$1 dedup $D: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dd/b.json') if l.startswith('{')][0]); n=d['nn']; print(round(d['value']), round(d['roofline']['frac'],4), round(n['share_of_step'],4), n['rows'], n['leaves'], round(n['rows_per_leaf'],4))")"
  done
done
