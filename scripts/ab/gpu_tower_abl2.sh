# As gpu_tower_abl.sh, alternating two libraries (LIBS) for each code.
set -u
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for code in ${CODES}; do
  for lib in ${LIBS}; do
    SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$lib SPMCTS_TOWER_CG=$code timeout -k 10 120 python scripts/bench_tower.py --trunk-only --iters ${ITERS:-10} --batch ${BATCH:-1536} > gpurun_out/abl/one.json 2> gpurun_out/abl/err.txt
    rc=$?
    if [ $rc -ne 0 ]; then echo "code $code lib $lib rc=$rc"; tail -3 gpurun_out/abl/err.txt; exit $rc; fi
    echo "$lib $(cat gpurun_out/abl/one.json)" >> gpurun_out/abl/abl2.txt
  done
done
cat gpurun_out/abl/abl2.txt
