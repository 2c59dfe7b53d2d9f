# Same-box A/B of two source trees (the previous commit in ab_prev/, a git worktree, vs this one): the
# tower tests of this tree, then alternating bench runs.  BENCH_ARGS selects the regime.
set -u
mkdir -p gpurun_out/dab
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_tower.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/dab/tower_tests.log 2>&1
rc=$?; tail -1 gpurun_out/dab/tower_tests.log; if [ $rc -ne 0 ]; then grep -E "^E |Error" gpurun_out/dab/tower_tests.log | head -10; exit $rc; fi
for rep in 1 2 3; do
  for d in ab_prev .; do
    (cd $d && timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > /tmp/dab.json 2> /tmp/dab.err) || { tail -3 /tmp/dab.err; exit 1; }
    echo "$d: $(python3 -c "import json; d=json.loads([l for l in open('/tmp/dab.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us']), round(d['nn']['share_of_step'],4))")"
  done
done
