# Where the trunk kernel's wave cycles go (one PMC pass, 8 SQ counters + GRBM): parked on
# s_waitcnt / barrier (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY, of which LDS issue
# SQ_WAIT_INST_LDS), issuing (SQ_ACTIVE_INST_ANY); LDS bank-conflict cycles against all LDS cycles.
set -u
mkdir -p gpurun_out/stall
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_tower" -f csv -d gpurun_out/stall/p1 -o run -- \
  python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 1536 > gpurun_out/stall/p1.json 2> gpurun_out/stall/p1.err
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/stall/p1.err; exit $rc; fi
python3 scripts/tower_util.py gpurun_out/stall/p1/run_counter_collection.csv gpurun_out/stall/tower_stall.json
