# Round 5: steady-state kernel trace of the driver-form bench on the final tree (42 warm-up plies, 7 traced)
# and its tower-free windows (scripts/trace_idle.py), as round 4's gpu_r04b.sh.
set -u
export TMPDIR=/tmp
O=gpurun_out/steady5
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d /tmp/steady5_trace -o run -- \
  python3 bench.py --warmup 42 --steps 7 --no-cpu-baseline --twin-no-dedup 0 --no-secondary > $O/bench_traced.json 2> $O/trace.err
rc=$?; echo "steady trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 scripts/trace_idle.py /tmp/steady5_trace/run_kernel_trace.csv 7 2 > $O/trace_idle.json && cat $O/trace_idle.json
rm -rf /tmp/steady5_trace
exit 0
