# Round-3 GPU pass 2: the whole -m gpu suite (statistical tests included), then a same-box bf16 / fp16
# bench A/B (alternated) and the train_model throughput line.  Own time limit per step.
set -u
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
O=gpurun_out/r03b
timeout -k 10 ${T:-1000} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 400 --timeout-method thread ${PYARGS:-} > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" $O/gpu_tests.log | tail -5; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/gpu_tests.log | head -80; exit $rc; }
for i in 1 2; do
  for dt in bf16 fp16; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --dtype $dt --no-cpu-baseline > $O/bench_${dt}_$i.json 2> $O/bench_${dt}_$i.err || exit $?
    python -c "import json; d=json.load(open('$O/bench_${dt}_$i.json')); print('$dt', $i, round(d['value']), round(d['roofline']['frac'],4))"
  done
done
if [ "${SKIP_TRAIN:-0}" != 1 ]; then
timeout -k 10 600 python -u scripts/bench_train.py > $O/train.json 2> $O/train.err
rc=$?; echo "train rc=$rc"; cut -c1-1500 $O/train.json; [ $rc -eq 0 ] || { tail -20 $O/train.err; exit $rc; }
fi
exit 0
