# (A/B code 1612 and the per-pair B pipeline were removed after this measurement: profiles/r05/m16_ablation/)
# Round 5: the C = 128 trunk on 12-board one-buffer 16x16x32 tiles (tower_wide16.h, A/B code 1612: each weight
# fragment for 16 MFMAs) -- bit-equality with the shipped two-buffer trunk (1602 = the product schedule in the
# A/B library), then trunk-only timing 6,144 boards bf16, alternated.
set -u
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
for c in 1602 1612; do
  SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/eq_$c.npz 32 bf16 > $O/eq_$c.log 2>&1 || { tail -5 $O/eq_$c.log; exit 1; }
done
python3 scripts/tower_code_equal.py cmp $O/eq_1602.npz $O/eq_1612.npz | tee -a $O/summary.txt
for rep in 1 2 3; do
  for c in 1602 1612; do
    SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 32 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c128 trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
exit 0
