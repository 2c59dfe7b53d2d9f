# Round 6: the trunk's L2<->fabric bytes for the traffic-cost A/B of scripts/gpu_r06h.sh (the shipped 16x16x32
# trunk, A/B code 1602, vs every layer on layer 0's weights, code 1665; trunk-only, 6,144 boards, bf16): FETCH_SIZE
# and WRITE_SIZE in their own rocprofv3 passes per code, then the two codes' times alternated once more.
set -u
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
export SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
BT="scripts/bench_tower.py --trunk-only --batch 6144 --ff 32 --iters 10"
for c in 1602 1665; do
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    SPMCTS_TOWER_CG=$c timeout -s KILL 180 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d $O/p${c}_$i -o run -- \
      python3 $BT > $O/p${c}_$i.json 2> $O/p${c}_$i.err
    rc=$?; echo "code $c pmc pass $i rc=$rc ($set)"; [ $rc -eq 0 ] || { tail -5 $O/p${c}_$i.err; exit $rc; }
  done
  python3 scripts/pmc_traffic.py $O/p${c}_1/run_counter_collection.csv $O/p${c}_2/run_counter_collection.csv \
    $O/traffic_$c.json 1 10 k_tower > $O/traffic_$c.out 2>&1 || { cat $O/traffic_$c.out; exit 1; }
  cut -c1-300 $O/traffic_$c.out | sed "s/^/code $c traffic: /" | tee -a $O/summary.txt
  rm -f $O/p${c}_*/run_counter_collection.csv
done
for rep in 1 2; do
  for c in 1602 1665; do
    SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 $BT > $O/one.json 2> $O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
exit 0
