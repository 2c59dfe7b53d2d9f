# Round 6: what the C = 128 trunk's fabric traffic costs.  The shipped 16x16x32 trunk
# (A/B code 1602, bf16, the product schedule) against the same kernel with every layer streaming layer 0's
# weights (code 1665: an L2-resident 295 KB weight set; wrong results by design), trunk-only, 6,144 boards,
# same box: time alternated x3, then per code FETCH_SIZE, WRITE_SIZE and clock / MFMA busy in their own
# rocprofv3 PMC passes.  Before that, the cross-lane dedup tests.
set -u
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
# first the cross-lane dedup cases (the recycled-store case with a 96-block store)
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -k "cross_lane" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|rows/leaf" $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A30 "Error" $O/tests.log | head -60; exit $rc; }
export SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
BT="scripts/bench_tower.py --trunk-only --batch 6144 --ff 32 --iters 10"
for rep in 1 2 3; do
  for c in 1602 1665; do
    SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 $BT > $O/one.json 2> $O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
for c in 1602 1665; do
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"; do
    i=$((i+1))
    SPMCTS_TOWER_CG=$c timeout -s KILL 180 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d $O/p${c}_$i -o run -- \
      python3 $BT > $O/p${c}_$i.json 2> $O/p${c}_$i.err
    rc=$?; echo "code $c pmc pass $i rc=$rc ($set)"; [ $rc -eq 0 ] || { tail -5 $O/p${c}_$i.err; exit $rc; }
  done
  python3 scripts/pmc_traffic.py $O/p${c}_1/run_counter_collection.csv $O/p${c}_2/run_counter_collection.csv \
    $O/traffic_$c.json 1 10 k_tower | cut -c1-300 | sed "s/^/code $c traffic: /" | tee -a $O/summary.txt
  python3 scripts/tower_util.py $O/p${c}_3/run_counter_collection.csv $O/util_$c.json 10 | cut -c1-260 \
    | sed "s/^/code $c util: /" | tee -a $O/summary.txt
  rm -f $O/p${c}_*/run_counter_collection.csv
done
exit 0
