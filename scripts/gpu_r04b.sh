# Round 4 GPU pass b: the C = 256 residual-scratch probes (gpu_c256_rsrc_probe.sh), then a steady-state
# kernel trace of the bench (42 warm-up plies, 7 traced) with its tower-free windows by ply phase
# (scripts/trace_idle.py).  Own time limit per step; the first failure ends the call.
set -u
export TMPDIR=/tmp
if [ "${SKIP_PROBE:-0}" != 1 ]; then bash scripts/gpu_c256_rsrc_probe.sh || exit 1; fi
O=gpurun_out/steady4
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- \
  python3 bench.py --warmup 42 --steps 7 --no-cpu-baseline --twin-no-dedup 0 --no-secondary > $O/bench_traced.json 2> $O/trace.err
rc=$?; echo "steady trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 scripts/trace_idle.py $O/trace/run_kernel_trace.csv 7 2 > $O/trace_idle.json && cat $O/trace_idle.json
gzip -f $O/trace/run_kernel_trace.csv
exit 0
