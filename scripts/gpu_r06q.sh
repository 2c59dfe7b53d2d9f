# Round 6: the evaluation cache as 64-byte records probed with plain loads (a candidate confirmed after an acquire
# fence) vs the previous layout (three arrays, every tag loaded with acquire; ab_libs/libspmcts_r06prev.so, built
# from commit acc0138's spmcts.hip with this tree's tower / trainconv objects).  Cache and dedup tests first, then
# the driver's form alternated twice, then the kernel stats of the new form.
set -u
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "eval_cache or dedup" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|rows/leaf" $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],1), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'cache_rows', d['nn']['cache_rows'], 'nn_share', round(d['nn']['share_of_step'],4))" "$1" "$2"; }
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
for rep in 1 2; do
  SPMCTS_LIB=$PWD/ab_libs/libspmcts_r06prev.so timeout -k 10 300 python3 bench.py $ARGS > $O/prev_$rep.json 2> $O/prev_$rep.err || { tail -20 $O/prev_$rep.err; exit 1; }
  line $O/prev_$rep.json "prev layout rep $rep:" | tee -a $O/summary.txt
  timeout -k 10 300 python3 bench.py $ARGS > $O/new_$rep.json 2> $O/new_$rep.err || { tail -20 $O/new_$rep.err; exit 1; }
  line $O/new_$rep.json "records rep $rep:" | tee -a $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py $ARGS > $O/traced.json 2> $O/trace.err
rc=$?; echo "trace rc=$rc" | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 scripts/trace_idle.py $O/trace/run_kernel_trace.csv 18 2 > $O/trace_idle.json && python3 -c "import json; d=json.load(open('$O/trace_idle.json')); print('tower-free', d['tower_free_frac'], d['by_phase_frac'])" | tee -a $O/summary.txt
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv && rm -f $O/trace/run_kernel_trace.csv
exit 0
