set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 1 ]; then tail -40 gpurun_out/gpu_tests.log; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; tail -3 gpurun_out/bench_full.err
exit $rc
