# Co-resident linear-heads kernel: tower/heads GPU tests, then same-box bench A/B against the
# LDS-staged kernel (SPMCTS_HEADS=lds) in the driver's short form and in steady state.
set -u
mkdir -p gpurun_out/hab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hab/tower_tests.log 2>&1
rc=$?; tail -1 gpurun_out/hab/tower_tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/hab/tower_tests.log | head; exit $rc; fi
for W in "5 20" "24 40"; do
  set -- $W
  for H in lds co lds co; do
    SPMCTS_HEADS=$H timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/hab/b.json 2>gpurun_out/hab/err.txt || { tail -3 gpurun_out/hab/err.txt; exit 1; }
    echo "bench w$1 heads $H: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/hab/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
  done
done
