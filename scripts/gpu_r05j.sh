# Round 5: the 4 x 1 wave plan of the 16x16x32 trunk (A/B codes 1640 / 1644) against the shipped 2 x 2 plan
# (1602), bf16, trunk-only; and the product library after the tower_m16.h generalisation against round 4's
# library (bit-equality, fp16 and bf16).
set -u
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
for dt in fp16 bf16; do
  SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts.so timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/eq_new_$dt.npz 32 $dt > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  SPMCTS_LIB=$PWD/ab_libs/libspmcts_r04.so timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/eq_old_$dt.npz 32 $dt >> $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  echo "product vs r04 $dt: $(python3 scripts/tower_code_equal.py cmp $O/eq_new_$dt.npz $O/eq_old_$dt.npz)" | tee -a $O/summary.txt
done
SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so CODES="1602 1640 1644" BATCHES="1536 6144" bash scripts/gpu_codes_ab.sh | tee -a $O/summary.txt
exit 0
