# Round 5: where a threaded tree kernel's sim spends its cycles (make prof: shader-clock marks per phase in
# sim_vl, libspmcts_prof.so), with and without the LDS block copies, on steady-state trees (bench_tree).
set -u
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
PROF=$PWD/self_play_reinforcement_learning_amd/libspmcts_prof.so
for c in 1 0; do
  SPMCTS_LIB=$PROF SPMCTS_TREE_COPIES=$c timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 --prof > $O/prof_$c.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  echo "copies=$c: $(tail -1 $O/prof_$c.json)" | tee -a $O/summary.txt
done
exit 0
