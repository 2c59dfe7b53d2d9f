set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k threaded > gpurun_out/vl_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_tests_all.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_k1.json 2> gpurun_out/bench_k1.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --search-threads 4 > gpurun_out/bench_k4.json 2> gpurun_out/bench_k4.err
