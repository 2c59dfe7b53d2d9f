set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --games 1024 --no-cpu-baseline > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc=$?
echo "bench small rc=$rc"; cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench full rc=$rc"; cat gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err
exit $rc
