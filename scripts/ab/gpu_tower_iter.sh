# Tower kernel iteration: correctness, micro-benchmark, end-to-end bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_tower.py -x -q > gpurun_out/tower_tests.log 2>&1
rc=$?; echo "tower tests rc=$rc"; tail -15 gpurun_out/tower_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_tower.py > gpurun_out/tower_bench.json 2> gpurun_out/tower_bench.err
rc=$?; echo "tower bench rc=$rc"; cat gpurun_out/tower_bench.json
if [ $rc -ne 0 ]; then tail -5 gpurun_out/tower_bench.err; exit $rc; fi
timeout -k 10 300 python scripts/bench_tower.py --ff 64 > gpurun_out/tower_bench256.json 2>> gpurun_out/tower_bench.err
rc=$?; echo "tower bench256 rc=$rc"; cat gpurun_out/tower_bench256.json
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${FULL_BENCH:-1}" = "1" ]; then
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_iter.json; tail -3 gpurun_out/bench_iter.err
fi
exit $rc
