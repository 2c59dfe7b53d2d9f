set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/engine_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k4 -o k4 -- python3 bench.py --no-cpu-baseline --search-threads 4 --steps 4 --warmup 2 > gpurun_out/bench_k4_prof.json 2> gpurun_out/bench_k4_prof.err
