# Round-2 measurement pass on the default bench workload (K = 4, two lanes):
#  1. a long run (one game generation of warm-up, then >= 60 s timed);
#  2. rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes on k_tower (scripts/gpu_prof_bench.sh);
#  3. one PMC pass with the clock and MFMA-busy counters on the bench's k_tower_dyn dispatches.
set -u
mkdir -p gpurun_out/prof gpurun_out/util
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --warmup 24 --steps 260 --no-cpu-baseline > gpurun_out/bench_long.json 2> gpurun_out/bench_long.err
rc=$?; echo "long bench rc=$rc"; cut -c1-300 gpurun_out/bench_long.json; if [ $rc -ne 0 ]; then exit $rc; fi
LANES=2 PSTEPS=3 bash scripts/gpu_prof_bench.sh
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA \
  --kernel-include-regex "k_tower_dyn" -f csv -d gpurun_out/util/bench -o run -- \
  python3 bench.py --steps 2 --warmup 24 --no-cpu-baseline > gpurun_out/util/bench_pmc.json 2> gpurun_out/util/bench_pmc.err
rc=$?; echo "clock pmc rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/util/bench_pmc.err; exit $rc; fi
python3 scripts/tower_util.py gpurun_out/util/bench/run_counter_collection.csv gpurun_out/util/tower_util_bench.json \
  $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/util/bench_pmc.json') if l.startswith('{')][0]); print(d['roofline']['dispatches'])")
