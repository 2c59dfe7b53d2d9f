# Tower kernel ablation timings (trunk only, SPMCTS_TOWER_CG codes, see csrc/tower.hip Cfg::ABL).
set -u
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for code in ${CODES:-2 11 100 101 102 104 108 116 124}; do
  SPMCTS_TOWER_CG=$code timeout -k 10 120 python scripts/bench_tower.py --trunk-only --iters ${ITERS:-10} --batch ${BATCH:-1536} >> gpurun_out/abl/abl.jsonl 2> gpurun_out/abl/err_$code.txt
  rc=$?
  if [ $rc -ne 0 ]; then echo "code $code rc=$rc"; tail -3 gpurun_out/abl/err_$code.txt; exit $rc; fi
done
cat gpurun_out/abl/abl.jsonl
