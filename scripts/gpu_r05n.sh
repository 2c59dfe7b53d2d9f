# Round 5: per-launch LDS copies of the child blocks in the threaded tree kernels (BlockCache: levels read
# LDS, no fence between sims).  (1) The bit-exact threaded parity tests and the engine tests; (2) Philox-mode
# games identical to round 4's library (scripts/rng_equal.py); (3) isolated tree kernels on steady-state
# trees, alternated with round 4's library; (4) the driver-form bench, alternated.
set -u
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r04.so
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 600 --timeout-method thread -k "not full_size and not spawns and not scheduler" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -100; exit $rc; }
fi
SPMCTS_LIB=$NEW timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_new.npz > $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
SPMCTS_LIB=$OLD timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_old.npz >> $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
python3 scripts/rng_equal.py --compare $O/rng_new.npz $O/rng_old.npz | tee -a $O/summary.txt
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 > $O/iso_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "iso steady $v: $(python3 -c "import json; d=json.loads(open('$O/iso_${v}_$rep.json').read().strip().splitlines()[-1]); print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k in ('select_avg_us', 'expand_avg_us', 'ply_ms', 'mean_levels')})")" | tee -a $O/summary.txt
  done
done
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 > $O/b_${v}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['tree_roofline']['avg_launch_us'],1), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
exit 0
