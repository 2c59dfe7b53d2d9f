# Round-1 profiling: kernel trace + stats of the bench, then HBM counters for k_select (separate passes).
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_traced.json 2> gpurun_out/prof/trace.err
rc=$?; echo "trace rc=$rc"; tail -3 gpurun_out/prof/trace.err
if [ $rc -ne 0 ]; then exit $rc; fi
find gpurun_out/prof/trace -name "*stats*" | head
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_select" -f csv -d gpurun_out/prof/pmc_fetch -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_pmc1.json 2> gpurun_out/prof/pmc1.err
rc=$?; echo "pmc fetch rc=$rc"; tail -3 gpurun_out/prof/pmc1.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_select" -f csv -d gpurun_out/prof/pmc_write -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_pmc2.json 2> gpurun_out/prof/pmc2.err
rc=$?; echo "pmc write rc=$rc"; tail -3 gpurun_out/prof/pmc2.err
exit $rc
