# Round 6, final tree: the profile bundle of the driver's command (scripts/gpu_r06l.sh), then the kernel stats of
# the same command with the evaluation cache off (--eval-cache 0), for the small kernels' durations beside it.
set -u
bash scripts/gpu_r06l.sh || exit 1
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace0 -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0 --eval-cache 0 > $O/traced_w0.json 2> $O/trace0.err
rc=$?; echo "trace w0 rc=$rc" | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -5 $O/trace0.err; exit $rc; }
cp $O/trace0/run_kernel_stats.csv $O/kernel_stats_w0.csv && rm -f $O/trace0/run_kernel_trace.csv
exit 0
