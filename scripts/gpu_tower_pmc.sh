# PMC counters for k_tower (one counter set per pass).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_]*\|TCC_[A-Z_a-z]*\|GRBM_[A-Z_]*\|TCP_[A-Z_]*" gpurun_out/pmc/counters_list.txt | sort -u > gpurun_out/pmc/names.txt
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d gpurun_out/pmc/p$i -o run -- \
     python3 scripts/bench_tower.py --iters 3 > gpurun_out/pmc/out$i.json 2> gpurun_out/pmc/err$i.txt
  rc=$?; echo "pass $i rc=$rc ($set)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/err$i.txt; fi
  if [ $rc -gt 1 ] && [ $rc -ne 255 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
