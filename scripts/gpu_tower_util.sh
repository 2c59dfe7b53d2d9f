# MFMA utilisation and clock of the shipped trunk kernel (trunk-only micro-benchmark, one
# 1,536-board launch per iteration = one full round of 6-board tiles): one PMC pass with
# GRBM_GUI_ACTIVE and the MFMA counters, reduced per dispatch by scripts/tower_util.py.
set -u
mkdir -p gpurun_out/util
export TMPDIR=/tmp
# DTYPES="bf16 fp16": one pass per element type of the trunk (BATCH boards per launch, default 1,536)
for dt in ${DTYPES:-bf16}; do
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_tower" -f csv -d gpurun_out/util/p_$dt -o run -- \
  python3 scripts/bench_tower.py --trunk-only --iters 10 --batch ${BATCH:-1536} --dtype $dt > gpurun_out/util/p_$dt.json 2> gpurun_out/util/p_$dt.err
rc=$?; echo "pmc $dt rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/util/p_$dt.err; exit $rc; fi
python3 scripts/tower_util.py gpurun_out/util/p_$dt/run_counter_collection.csv gpurun_out/util/tower_util_$dt.json
done
