# Trunk timing for a list of "tag:code" pairs (SPMCTS_TOWER_CG code; the tag is only echoed).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/tower_codes.jsonl
for fc in ${PAIRS}; do
  form=${fc%%:*}; code=${fc##*:}
  SPMCTS_TOWER_CG=$code timeout -k 10 120 python scripts/bench_tower.py --trunk-only --iters 30 --batch ${BATCH:-4096} > gpurun_out/one.json 2> gpurun_out/tb.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$fc rc=$rc"; tail -5 gpurun_out/tb.err; exit $rc; fi
  echo "{\"form\": $form, \"r\": $(cat gpurun_out/one.json)}" | tee -a gpurun_out/tower_codes.jsonl
done
