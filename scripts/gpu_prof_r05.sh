# Round-5 profile bundle of the current tree (same steps as gpu_prof_r04.sh), one box: rocprofv3 kernel trace (--stats) + FETCH_SIZE /
# WRITE_SIZE passes of the bench's trunk (scripts/gpu_prof_bench.sh, the bench defaults: fp16 trunk), the
# tree kernels' FETCH/WRITE_SIZE (gpu_prof_tree.sh), and one in-bench PMC pass with the clock and MFMA-busy
# counters on the timed k_tower_dyn dispatches (scripts/tower_util.py; fp16, then bf16).
# Each step has its own time limit; the first failure ends the call.
set -u
export TMPDIR=/tmp
if [ "${SKIP_TRACE:-0}" != 1 ]; then
bash scripts/gpu_prof_bench.sh || exit $?
bash scripts/gpu_prof_tree.sh || exit $?
fi
mkdir -p gpurun_out/util
for dt in ${DTYPES:-fp16 bf16}; do
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    --kernel-include-regex "k_tower_dyn" -f csv -d gpurun_out/util/bench_$dt -o run -- \
    python3 bench.py --steps 3 --warmup 24 --dtype $dt --no-cpu-baseline --twin-no-dedup 0 --no-secondary \
    > gpurun_out/util/bench_pmc_$dt.json 2> gpurun_out/util/bench_pmc_$dt.err
  rc=$?; echo "clock pmc $dt rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/util/bench_pmc_$dt.err; exit $rc; fi
  python3 scripts/tower_util.py gpurun_out/util/bench_$dt/run_counter_collection.csv gpurun_out/util/tower_util_bench_$dt.json \
    $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/util/bench_pmc_$dt.json') if l.startswith('{')][0]); print(d['roofline']['dispatches'])")
  rm -f gpurun_out/util/bench_$dt/run_counter_collection.csv
  cat gpurun_out/util/tower_util_bench_$dt.json | head -c 400; echo
done
# one PMC pass of the driver's own bench command (--warmup 5 --steps 20) over the kernels beside the trunk:
# per-kernel clock, MFMA busy and wave-cycle split (scripts/pmc_per_kernel.py; the profiler serialises them)
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex "k_tower_dyn|k_expand_vl|k_heads_co|k_scan_need|k_select_vl" -f csv -d gpurun_out/util/driver -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 > gpurun_out/util/driver_pmc.json 2> gpurun_out/util/driver_pmc.err
rc=$?; echo "driver-form per-kernel pmc rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/util/driver_pmc.err; exit $rc; fi
python3 scripts/pmc_per_kernel.py gpurun_out/util/driver/run_counter_collection.csv gpurun_out/util/driver_per_kernel.json
rm -f gpurun_out/util/driver/run_counter_collection.csv
exit 0
