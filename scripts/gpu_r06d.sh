# Round 6, fourth pass (the final tree):
#  (0) the cross-lane / dedup engine tests; the peer push on the follower's push stream vs on the leader's
#      stream (A/B library, SPMCTS_PEER_PUSH=leader), alternated;
#  (1) lane split A/B with cross-lane dedup (lane 0's share 0.5 / 0.48 / 0.46), alternated;
#  (2) the profile bundle of the driver's command (--warmup 5 --steps 20, same seeds; CPU leg and no-dedup twin
#      off so the trace's last dispatches are the timed region): kernel trace + stats, trace-recomputed roofline,
#      trunk FETCH_SIZE / WRITE_SIZE, trunk clock / MFMA busy, tree-kernel FETCH_SIZE / WRITE_SIZE;
#  (3) the tower-free windows of the traced run (scripts/trace_idle.py).
set -u
O=gpurun_out/r06d
P=$O/prof
mkdir -p $O $P
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0"
val() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['rows_per_leaf'],4), round(d['nn']['share_of_step'],4), d['config'].get('lane_games'), round(d['roofline']['clock']['clock_ghz'],3))" "$1"; }
ndisp() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d['roofline']['dispatches'])" "$1"; }
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "cross_lane or leaf_dedup or laned" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -80; exit $rc; }
for rep in 1 2; do
  for v in stream leader; do
    if [ $v = leader ]; then export SPMCTS_PEER_PUSH=leader; else unset SPMCTS_PEER_PUSH; fi
    SPMCTS_LIB=$AB timeout -k 10 300 python3 bench.py $ARGS > $O/p_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench push on $v (A/B lib): $(val $O/p_${v}_$rep.json)" | tee -a $O/summary.txt
  done
done
unset SPMCTS_PEER_PUSH
for rep in 1 2; do
  for sh in 0.5 0.48 0.46; do
    timeout -k 10 300 python3 bench.py $ARGS --lane0-share $sh > $O/b_${sh}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench share $sh: $(val $O/b_${sh}_$rep.json)" | tee -a $O/summary.txt
  done
done
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
