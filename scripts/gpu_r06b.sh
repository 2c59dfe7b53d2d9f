# Round 6, second pass: deferred all-terminal fills (fill_tree_vl) and the lock-step issue order of the lanes
# (every lane's network, then the followers' leader-served rows, then the expands).
#  (1) bit-exact parity + engine tests (threaded / sequential, cross-lane dedup), Philox games identical to round
#      5's library (scripts/rng_equal.py), isolated steady-state tree kernels alternated with round 5's library;
#  (2) driver-form bench: this tree with cross-lane dedup on / off and round 5's library, alternated;
#  (3) the config-3 search-shift bound and its control (ResNet-256x20, 800 sims);
#  (4) the Winograd MFMA / vector-issue probe (scripts/diag/mfma_valu_probe.hip, built here).
set -u
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r05.so
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0"
val() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['rows_per_leaf'],4), round(d['nn']['share_of_step'],4), d['config'].get('cross_lane_dedup'), round(d['roofline']['clock']['clock_ghz'],3) if d['roofline'].get('clock') and d['roofline']['clock'].get('clock_ghz') else None)" "$1"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "not full_size and not spawns and not scheduler and not bench_line" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -100; exit $rc; }
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
  for v in cross nocross old; do
    X=""; LIB=$NEW
    [ $v = nocross ] && X="--no-cross-dedup"
    [ $v = old ] && { X="--no-cross-dedup"; LIB=$OLD; }
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 bench.py $ARGS $X > $O/b_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(val $O/b_${v}_$rep.json)" | tee -a $O/summary.txt
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_statistical.py -m gpu -x -q -s --timeout 600 --timeout-method thread \
  -k "config3" > $O/c256.log 2>&1
rc=$?; grep -E "config3|passed|failed" $O/c256.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -30 $O/c256.log; exit $rc; }
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize scripts/diag/mfma_valu_probe.hip -o $O/mfma_valu_probe > $O/probe_build.log 2>&1 || { tail -5 $O/probe_build.log; exit 1; }
timeout -k 10 300 $O/mfma_valu_probe > $O/mfma_valu_probe.json 2> $O/probe.err || { tail -5 $O/probe.err; exit 1; }
cat $O/mfma_valu_probe.json | tee -a $O/summary.txt
rm -f $O/mfma_valu_probe
exit 0
