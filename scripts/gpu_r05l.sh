# Round 5: MFMA-shape clock probe on the C = 256 one-buffer trunk (A/B code 2308: each 32x32x16 as two 16x16x32,
# timing only) against the shipped form (2300), bf16, trunk-only, 6,144 boards, alternated; + a PMC clock pass.
set -u
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
for rep in 1 2 3; do
  for c in 2300 2308; do
    SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 64 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c256 trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
for c in 2300 2308; do
  SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_tower" -f csv -d $O/p_$c -o run -- \
    python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 6144 --ff 64 > $O/p.json 2> $O/p.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $O/p.err; exit $rc; fi
  python3 scripts/tower_util.py $O/p_$c/run_counter_collection.csv $O/util_$c.json > /dev/null
  rm -f $O/p_$c/run_counter_collection.csv
  echo "pmc $c: $(python3 -c "import json; d=json.load(open('$O/util_$c.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a $O/summary.txt
done
exit 0
