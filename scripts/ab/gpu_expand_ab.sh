# GPU suite on the current build, then same-box A/B of two library builds: isolated tree kernels
# (scripts/bench_tree.py) and the bench in the driver's short form and in steady state.
# LIBS="prev.so new.so" (in self_play_reinforcement_learning_amd/).
set -u
mkdir -p gpurun_out/xab
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/xab/gpu_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/xab/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/xab/gpu_tests.log | head -20; exit $rc; fi
fi
for rep in 1 2; do
  for lib in ${LIBS}; do
    SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$lib timeout -k 10 120 python3 scripts/bench_tree.py > gpurun_out/xab/iso.json 2>gpurun_out/xab/err.txt || { tail -3 gpurun_out/xab/err.txt; exit 1; }
    echo "iso $lib: $(python3 -c "import json; d=json.loads(open('gpurun_out/xab/iso.json').read().strip().splitlines()[-1]); print(round(d['select_avg_us'],1), round(d['expand_avg_us'],1))")"
  done
done
for W in "5 20" "24 40"; do
  set -- $W
  for rep in 1 2; do
    for lib in ${LIBS}; do
      SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$lib timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/xab/b.json 2>gpurun_out/xab/err.txt || { tail -3 gpurun_out/xab/err.txt; exit 1; }
      echo "bench w$1 $lib: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/xab/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
    done
  done
done
