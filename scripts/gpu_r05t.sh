# Round 5: the Philox block window in the threaded tree kernels (a group's 8 computed blocks serve the next
# level when they hold its draws): (1) threaded parity + engine tests, (2) Philox games vs round 4's library,
# (3) isolated tree kernels vs the previous commit's library (DPP reductions), alternated.
set -u
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r05dpp.so
R04=$PWD/ab_libs/libspmcts_r04.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 600 --timeout-method thread -k "not full_size and not spawns and not scheduler" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -100; exit $rc; }
SPMCTS_LIB=$NEW timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_new.npz > $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
SPMCTS_LIB=$R04 timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_old.npz >> $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
python3 scripts/rng_equal.py --compare $O/rng_new.npz $O/rng_old.npz | tee -a $O/summary.txt
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 > $O/iso_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "iso steady $v: $(python3 -c "import json; d=json.loads(open('$O/iso_${v}_$rep.json').read().strip().splitlines()[-1]); print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k in ('select_avg_us', 'expand_avg_us', 'ply_ms', 'mean_levels')})")" | tee -a $O/summary.txt
  done
done
exit 0
