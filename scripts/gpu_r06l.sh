# Round 6, the profile bundle of the driver's command with the evaluation cache on (window 1, bench.py's default);
# otherwise as scripts/gpu_r06f.sh:
#  (2) the profile bundle of the driver's command (--warmup 5 --steps 20, same seeds; CPU leg and no-dedup twin
#      off so the trace's last dispatches are the timed region): kernel trace + stats, trace-recomputed roofline,
#      trunk FETCH_SIZE / WRITE_SIZE, trunk clock / MFMA busy, tree-kernel FETCH_SIZE / WRITE_SIZE;
#  (3) the tower-free windows of the traced run (scripts/trace_idle.py).
set -u
O=gpurun_out/r06l
P=$O/prof
mkdir -p $O $P
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
val() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['rows_per_leaf'],4), round(d['nn']['share_of_step'],4), d['config'].get('lane_games'), round(d['roofline']['clock']['clock_ghz'],3))" "$1"; }
ndisp() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d['roofline']['dispatches'])" "$1"; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $P/trace -o run -- python3 bench.py $ARGS > $P/bench_traced.json 2> $P/trace.err
rc=$?; echo "trace rc=$rc" | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -5 $P/trace.err; exit $rc; }
python3 scripts/roofline_from_trace.py $P/bench_traced.json $P/trace/run_kernel_trace.csv $P/roofline_from_trace.json | cut -c1-700 | tee -a $O/summary.txt
python3 scripts/tower_union.py $P/trace/run_kernel_trace.csv 2 $P/k_tower_union.json $(ndisp $P/bench_traced.json) > /dev/null
python3 scripts/trace_idle.py $P/trace/run_kernel_trace.csv 18 2 > $P/trace_idle.json && head -c 600 $P/trace_idle.json | tee -a $O/summary.txt; echo
cp $P/trace/run_kernel_stats.csv $P/kernel_stats.csv
gzip -c $P/trace/run_kernel_trace.csv > $P/run_kernel_trace.csv.gz && rm -f $P/trace/run_kernel_trace.csv
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d $P/pmc$i -o run -- \
     python3 bench.py $ARGS > $P/pmc$i.json 2> $P/pmc$i.err
  rc=$?; echo "trunk pmc pass $i rc=$rc ($set)"; [ $rc -eq 0 ] || { tail -5 $P/pmc$i.err; exit $rc; }
done
python3 scripts/pmc_traffic.py $P/pmc1/run_counter_collection.csv $P/pmc2/run_counter_collection.csv $P/k_tower_traffic.json 2 \
  $(ndisp $P/pmc1.json) | tee -a $O/summary.txt
rm -f $P/pmc1/run_counter_collection.csv $P/pmc2/run_counter_collection.csv
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    --kernel-include-regex "k_tower_dyn" -f csv -d $P/util -o run -- python3 bench.py $ARGS > $P/util.json 2> $P/util.err
rc=$?; echo "util pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/util.err; exit $rc; }
python3 scripts/tower_util.py $P/util/run_counter_collection.csv $P/tower_util_bench_fp16.json $(ndisp $P/util.json) | cut -c1-400 | tee -a $O/summary.txt
rm -f $P/util/run_counter_collection.csv
T=$O/tree
mkdir -p $T
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "k_select_vl|k_expand_vl" -f csv -d $T/pmc$i -o run -- \
     python3 bench.py $ARGS > $T/pmc$i.json 2> $T/pmc$i.err
  rc=$?; echo "tree pmc pass $i rc=$rc ($set)"; [ $rc -eq 0 ] || { tail -5 $T/pmc$i.err; exit $rc; }
done
python3 scripts/pmc_tree.py $T/pmc1/run_counter_collection.csv $T/pmc2/run_counter_collection.csv $T/tree_traffic.json \
  $(python3 -c "import json; d=json.loads([l for l in open('$T/pmc1.json') if l.startswith('{')][0]); print(d['tree_roofline']['launches'])") | tee -a $O/summary.txt
rm -f $T/pmc1/run_counter_collection.csv $T/pmc2/run_counter_collection.csv
exit 0
