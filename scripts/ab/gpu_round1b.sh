set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_tower.py -x -q > gpurun_out/tower_tests.log 2>&1
rc=$?; echo "tower tests rc=$rc"; tail -30 gpurun_out/tower_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_tower.py > gpurun_out/tower_bench.json 2> gpurun_out/tower_bench.err
rc=$?; echo "tower bench rc=$rc"; cat gpurun_out/tower_bench.json; tail -3 gpurun_out/tower_bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_tower.py --ff 64 --batch 4096 > gpurun_out/tower_bench256.json 2>> gpurun_out/tower_bench.err
rc=$?; echo "tower bench256 rc=$rc"; cat gpurun_out/tower_bench256.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_full2.json 2> gpurun_out/bench_full2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full2.json; tail -3 gpurun_out/bench_full2.err
exit $rc
