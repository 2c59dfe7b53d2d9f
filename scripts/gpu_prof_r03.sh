# Round-3 profile bundle of the final tree, one box: rocprofv3 trace + FETCH/WRITE_SIZE of the bench's
# trunk (scripts/gpu_prof_bench.sh), the tree kernels' FETCH/WRITE_SIZE (gpu_prof_tree.sh), clock and
# MFMA busy of the bf16 and fp16 trunks (gpu_tower_util.sh), and the LDS-ring trunk vs the shipped trunk
# (trunk-only timings, alternated).  Each step has its own time limit; the first failure ends the call.
set -u
export TMPDIR=/tmp
bash scripts/gpu_prof_bench.sh || exit $?
bash scripts/gpu_prof_tree.sh || exit $?
DTYPES="bf16 fp16" BATCH=6144 bash scripts/gpu_tower_util.sh || exit $?
mkdir -p gpurun_out/ring
for BATCH in 1536 6144; do
  for rep in 1 2; do
    for ring in 0 1; do
      SPMCTS_TOWER_RING=$ring timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 > gpurun_out/ring/one.json 2> gpurun_out/ring/err.txt || { tail -3 gpurun_out/ring/err.txt; exit 1; }
      echo "trunk $BATCH ring $ring: $(python3 -c "import json; d=json.loads(open('gpurun_out/ring/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a gpurun_out/ring/ring_ab.txt
    done
  done
done
