# Round 6, first pass on the box:
#  (1) the tree-kernel change (fence only after issued stores; counters flushed on error paths): the bit-exact
#      threaded / sequential parity and engine tests, Philox games identical to round 5's library
#      (scripts/rng_equal.py), isolated steady-state tree kernels alternated with round 5's library;
#  (2) the driver's own bench command with the same-run clock (amdsmi), and once without the sampler; cross-lane
#      leaf dedup on / off alternated;
#  (3) the profile bundle of the driver's command (--warmup 5 --steps 20, same seeds; CPU leg and the
#      no-dedup twin off so the trace's last dispatches are the timed region): kernel trace + stats, the
#      trace-recomputed roofline of the same run, FETCH_SIZE / WRITE_SIZE passes, one clock / MFMA-busy pass.
set -u
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r05.so
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0"
line() { python3 -c "import json,sys; print([l for l in open(sys.argv[1]) if l.startswith('{')][0].strip())" "$1"; }
ndisp() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d['roofline']['dispatches'])" "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_trainconv.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "not full_size and not spawns and not scheduler and not bench_line" > $O/tests.log 2>&1
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
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
echo "driver: $(line $O/bench_driver.json | cut -c1-200)" | tee -a $O/summary.txt
python3 -c "import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][0]); r=d['roofline']; print('frac', r['frac'], 'executed', r['executed']['frac'], 'clock', r['clock'])" | tee -a $O/summary.txt
for rep in 1 2; do
  for v in cross nocross; do
    X=""; [ $v = nocross ] && X="--no-cross-dedup"
    timeout -k 10 300 python3 bench.py $ARGS $X > $O/b_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['rows_per_leaf'],4), round(d['nn']['share_of_step'],4), d['config']['cross_lane_dedup'])")" | tee -a $O/summary.txt
  done
done
timeout -k 10 300 python3 bench.py $ARGS --no-clock > $O/bench_noclock.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
timeout -k 10 300 python3 bench.py $ARGS > $O/bench_clock.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
echo "sampler A/B: off $(python3 -c "import json; print(round(json.loads([l for l in open('$O/bench_noclock.json') if l.startswith('{')][0])['value']))") on $(python3 -c "import json; print(round(json.loads([l for l in open('$O/bench_clock.json') if l.startswith('{')][0])['value']))")" | tee -a $O/summary.txt
# --- profile bundle of the driver's command
P=$O/prof
mkdir -p $P
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $P/trace -o run -- python3 bench.py $ARGS > $P/bench_traced.json 2> $P/trace.err
rc=$?; echo "trace rc=$rc" | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -5 $P/trace.err; exit $rc; }
python3 scripts/roofline_from_trace.py $P/bench_traced.json $P/trace/run_kernel_trace.csv $P/roofline_from_trace.json | cut -c1-600 | tee -a $O/summary.txt
python3 scripts/tower_union.py $P/trace/run_kernel_trace.csv 2 $P/k_tower_union.json $(ndisp $P/bench_traced.json) > /dev/null
cp $P/trace/run_kernel_stats.csv $P/kernel_stats.csv
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d $P/pmc$i -o run -- \
     python3 bench.py $ARGS > $P/pmc$i.json 2> $P/pmc$i.err
  rc=$?; echo "pmc pass $i rc=$rc ($set)"; [ $rc -eq 0 ] || { tail -5 $P/pmc$i.err; exit $rc; }
done
python3 scripts/pmc_traffic.py $P/pmc1/run_counter_collection.csv $P/pmc2/run_counter_collection.csv $P/k_tower_traffic.json 2 \
  $(ndisp $P/pmc1.json) | tee -a $O/summary.txt
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    --kernel-include-regex "k_tower_dyn" -f csv -d $P/util -o run -- python3 bench.py $ARGS > $P/util.json 2> $P/util.err
rc=$?; echo "util pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/util.err; exit $rc; }
python3 scripts/tower_util.py $P/util/run_counter_collection.csv $P/tower_util_bench_fp16.json $(ndisp $P/util.json) | cut -c1-400 | tee -a $O/summary.txt
rm -f $P/pmc1/run_counter_collection.csv $P/pmc2/run_counter_collection.csv $P/util/run_counter_collection.csv
exit 0
