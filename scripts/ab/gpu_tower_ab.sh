set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cg in ${CGS_TEST:-10 11}; do
SPMCTS_TOWER_CG=$cg timeout -k 10 600 python -m pytest tests/test_gpu_tower.py -x -q > gpurun_out/tower_tests_$cg.log 2>&1
rc=$?; echo "cg=$cg tower tests rc=$rc"; tail -2 gpurun_out/tower_tests_$cg.log
if [ $rc -ne 0 ]; then tail -30 gpurun_out/tower_tests_$cg.log; exit $rc; fi
done
for batch in ${BATCHES:-4096 3800}; do
for cg in ${CGS:-2 10 11 2 10 11}; do
  SPMCTS_TOWER_CG=$cg timeout -k 10 300 python scripts/bench_tower.py --iters 40 --batch $batch > gpurun_out/tb_cg$cg.json 2>/dev/null || exit 1
  echo "batch=$batch cg=$cg $(python -c "import json;d=json.load(open('gpurun_out/tb_cg$cg.json'));print(d['hip_trunk_only'], d['hip'])")"
done
done
