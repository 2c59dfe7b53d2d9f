# Round 5: where the threaded tree kernels' waves spend their cycles (rocprofv3 PMC, one pass per counter
# set, isolated tree kernels on steady-state trees via bench_tree.py).
set -u
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/avail.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
grep -o "SQ_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/sq_counters.txt || true
P=1
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "k_select_vl|k_expand_vl" -f csv -d /tmp/pmc_$P -o run -- \
    python3 scripts/bench_tree.py --warmup 24 --plies 1 > $O/p$P.json 2> $O/p$P.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $P rc=$rc"; tail -5 $O/p$P.err; exit $rc; fi
  python3 scripts/pmc_per_kernel.py /tmp/pmc_$P/run_counter_collection.csv $O/pmc_$P.json "k_select_vl|k_expand_vl" | tee -a $O/summary.txt
  rm -rf /tmp/pmc_$P
  P=$((P+1))
done
exit 0
