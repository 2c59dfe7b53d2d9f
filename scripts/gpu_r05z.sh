# (A/B code 1612 and the per-pair B pipeline were removed after this measurement: profiles/r05/m16_ablation/)
# Round 5: wide16 with the B operands pipelined per (k-step, tile) pair (tap_pairs: 0 spills at C = 256, was 9-20):
# (1) C = 256 outputs bit-equal to the previous product library (2 and 20 blocks, host + device-count paths, bf16
# and fp16); (2) the C = 128 12-board code 1612 bit-equal to the two-buffer trunk (1602); (3) trunk-only timing:
# C = 256 new vs previous library, and C = 128 1612 vs 1602, alternated.
set -u
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r05dpp.so
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
for dt in bf16 fp16; do
  SPMCTS_LIB=$NEW timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/c256_new_$dt.npz 64 $dt > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  SPMCTS_LIB=$OLD timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/c256_old_$dt.npz 64 $dt > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  echo "c256 $dt new vs previous: $(python3 scripts/tower_code_equal.py cmp $O/c256_new_$dt.npz $O/c256_old_$dt.npz)" | tee -a $O/summary.txt
done
for c in 1602 1612; do
  SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/eq_$c.npz 32 bf16 > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
done
echo "c128 1612 vs 1602: $(python3 scripts/tower_code_equal.py cmp $O/eq_1602.npz $O/eq_1612.npz)" | tee -a $O/summary.txt
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 64 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c256 trunk 6144 $v: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
  for c in 1602 1612; do
    SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 32 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c128 trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
exit 0
