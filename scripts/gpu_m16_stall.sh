# Stall / LDS PMC of the 16x16x32 C = 128 trunk (product library) and round 3's 32x32x16 trunk (A/B library,
# SPMCTS_TOWER_M16=0), trunk-only, 6,144 boards, fp16: wait shares, LDS bank conflicts, MFMA busy, clock.
set -u
O=gpurun_out/m16stall
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
for v in m16 old; do
  if [ $v = m16 ]; then E="SPMCTS_LIB=$L/libspmcts.so"; else E="SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_M16=0"; fi
  env $E timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_tower" -f csv -d $O/p_$v -o run -- \
    python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 6144 --dtype fp16 > $O/p.json 2> $O/p.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $O/p.err; exit $rc; fi
  python3 scripts/tower_util.py $O/p_$v/run_counter_collection.csv $O/stall_$v.json
  rm -f $O/p_$v/run_counter_collection.csv
  echo "pmc $v: $(python3 -c "import json; d=json.load(open('$O/stall_$v.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a $O/summary.txt
done
exit 0
