# Trunk variants of the A/B library (SPMCTS_TOWER_CG codes, C = 128 bf16 host path) against the shipped
# full-tile configuration (code 200), on one box: outputs bit for bit (scripts/tower_code_equal.py), one PMC
# pass each (clock, MFMA busy, waits: scripts/tower_util.py), trunk-only timings alternated.
# CODES="304 ..." (default 304: weight-major MFMA order).
set -u
O=gpurun_out/codes_clock
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
CODES=${CODES:-304}
SPMCTS_LIB=$AB SPMCTS_TOWER_CG=200 timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/c200.npz 32 || exit 1
for c in $CODES; do
  SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/c$c.npz 32 || exit 1
  echo "outputs $c vs 200: $(python3 scripts/tower_code_equal.py cmp $O/c200.npz $O/c$c.npz)" | tee -a $O/summary.txt
done
for c in 200 $CODES; do
  SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_tower" -f csv -d $O/p_$c -o run -- \
    python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 6144 > $O/p.json 2> $O/p.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $O/p.err; exit $rc; fi
  python3 scripts/tower_util.py $O/p_$c/run_counter_collection.csv $O/util_$c.json
  rm -f $O/p_$c/run_counter_collection.csv
  echo "pmc $c: $(python3 -c "import json; d=json.load(open('$O/util_$c.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a $O/summary.txt
done
for BATCH in 1536 6144; do
  for rep in 1 2 3; do
    for c in 200 $CODES; do
      SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
      echo "trunk $BATCH $c $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a $O/summary.txt
    done
  done
done
exit 0
