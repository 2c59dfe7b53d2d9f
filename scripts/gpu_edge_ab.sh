# Round 4: the conflict-free edge layout (tower_edge.h from scripts/edge_layout_model.py) against the
# round-3 library.  LIBS="old.so new.so" under self_play_reinforcement_learning_amd/.
#   1. trunk outputs bit-equal (scripts/tower_code_equal.py; bf16 and fp16);
#   2. tower + parity GPU tests on the new build;
#   3. one PMC pass per build (trunk-only, one round of 6-board tiles, both dtypes): LDS bank-conflict
#      cycles, waits, MFMA busy, clock (scripts/tower_util.py);
#   4. trunk-only timings (one and four rounds), both dtypes, alternated;
#   5. driver-form bench (warm-up 5, 20 plies), alternated, REPS rounds.
set -u
mkdir -p gpurun_out/edge
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
set -- $LIBS
A=$1; B=$2
for dt in bf16 fp16; do
  SPMCTS_LIB=$L/$A DT=$dt timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/edge/a_$dt.npz 32 $dt && \
  SPMCTS_LIB=$L/$B DT=$dt timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/edge/b_$dt.npz 32 $dt || exit 1
  python3 scripts/tower_code_equal.py cmp gpurun_out/edge/a_$dt.npz gpurun_out/edge/b_$dt.npz | tee -a gpurun_out/edge/summary.txt || exit 1
done
SPMCTS_LIB=$L/$B timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/edge/tests.log 2>&1
rc=$?; tail -1 gpurun_out/edge/tests.log | tee -a gpurun_out/edge/summary.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in $A $B; do
  for dt in bf16 fp16; do
    SPMCTS_LIB=$L/$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_tower" -f csv -d gpurun_out/edge/p_${lib%.so}_$dt -o run -- \
      python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 1536 --dtype $dt > gpurun_out/edge/p.json 2> gpurun_out/edge/p.err
    rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 gpurun_out/edge/p.err; exit $rc; fi
    python3 scripts/tower_util.py gpurun_out/edge/p_${lib%.so}_$dt/run_counter_collection.csv gpurun_out/edge/stall_${lib%.so}_$dt.json
    echo "pmc $lib $dt: $(python3 -c "import json; d=json.load(open('gpurun_out/edge/stall_${lib%.so}_$dt.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a gpurun_out/edge/summary.txt
  done
done
for BATCH in 1536 6144; do
  for dt in bf16 fp16; do
    for rep in 1 2; do
      for lib in $A $B; do
        SPMCTS_LIB=$L/$lib timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 --dtype $dt > gpurun_out/edge/one.json 2>gpurun_out/edge/err.txt || { tail -3 gpurun_out/edge/err.txt; exit 1; }
        echo "trunk $BATCH $dt $lib $(python3 -c "import json; d=json.loads(open('gpurun_out/edge/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a gpurun_out/edge/summary.txt
      done
    done
  done
done
for rep in $(seq ${REPS:-2}); do
  for lib in $A $B; do
    SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/edge/b_${lib%.so}_$rep.json 2>gpurun_out/edge/err.txt || { tail -3 gpurun_out/edge/err.txt; exit 1; }
    echo "bench w5 $lib: $(python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/edge/b_${lib%.so}_$rep.json') if l.startswith('{')][0])
print(d['dtype'], round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), 'twin', round(d.get('no_dedup_twin', {}).get('value', 0)), 'secondary', d.get('secondary_dtype', {}).get('dtype'), round(d.get('secondary_dtype', {}).get('value', 0)))")" | tee -a gpurun_out/edge/summary.txt
  done
done
