# Ring trunk (tower_ring.h) check + same-box A/B against the two-buffer trunk (SPMCTS_TOWER_RING=0):
# tower tests first (own limit), then the trunk micro-benchmark and the bench, alternated.
set -u
mkdir -p gpurun_out/ring
export TMPDIR=/tmp
O=gpurun_out/ring
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tower_tests.log 2>&1
rc=$?; echo "tower tests rc=$rc"; tail -3 $O/tower_tests.log; [ $rc -eq 0 ] || { grep -B3 -A25 "FAILED\|Error\|error" $O/tower_tests.log | head -60; exit $rc; }
for i in 1 2; do
  for ring in 1 0; do
    SPMCTS_TOWER_RING=$ring timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_ring${ring}_$i.json 2> $O/bench_ring${ring}_$i.err || { tail -5 $O/bench_ring${ring}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_ring${ring}_$i.json')); print('ring', $ring, $i, round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_dispatch_us'],1))"
  done
done
exit 0
