set -u
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof2/trace -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/bench_traced.json 2> gpurun_out/prof2/trace.err
rc=$?; echo "trace rc=$rc"; cat gpurun_out/prof2/bench_traced.json | cut -c1-300
exit $rc
