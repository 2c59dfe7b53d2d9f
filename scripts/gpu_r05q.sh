# Round 5: isolated threaded tree kernels, one tree per wave (SPMCTS_TREE_BLOCK=8) vs 8 trees per wave (64),
# with and without the LDS block copies (A/B library), steady-state trees.
set -u
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
for tb in 8 64; do
  for c in 1 0; do
    SPMCTS_LIB=$AB SPMCTS_TREE_BLOCK=$tb SPMCTS_TREE_COPIES=$c timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 > $O/iso_${tb}_$c.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "iso tb=$tb copies=$c: $(python3 -c "import json; d=json.loads(open('$O/iso_${tb}_$c.json').read().strip().splitlines()[-1]); print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k in ('select_avg_us', 'expand_avg_us', 'ply_ms')})")" | tee -a $O/summary.txt
  done
done
exit 0
