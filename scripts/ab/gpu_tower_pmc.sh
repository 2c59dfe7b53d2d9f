# PMC counters for the trunk kernel (one counter set per pass), for SPMCTS_TOWER_CG codes in CODES.
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for code in ${CODES:-2}; do
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  SPMCTS_TOWER_CG=$code timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d gpurun_out/pmc/c${code}_p$i -o run -- \
     python3 scripts/bench_tower.py --trunk-only --iters 3 --batch ${BATCH:-1536} > gpurun_out/pmc/out_${code}_$i.json 2> gpurun_out/pmc/err_${code}_$i.txt
  rc=$?; echo "code $code pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/err_${code}_$i.txt; fi
done
done
exit 0
