set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k threaded > gpurun_out/vl_tests4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --search-threads 4 > gpurun_out/bench_k4_wgfence.json 2> gpurun_out/bench_k4_wgfence.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k4b -o k4 -- python3 bench.py --no-cpu-baseline --search-threads 4 --steps 4 --warmup 2 > gpurun_out/bench_k4b_prof.json 2> gpurun_out/bench_k4b_prof.err
