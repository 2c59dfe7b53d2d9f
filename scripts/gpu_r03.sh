# Round-3 GPU pass: the whole -m gpu suite, the bench (driver form), and the --gpus N self-launch:
# a 2-rank rehearsal on the box's one GPU (gloo, oversubscription allowed) and the refusal of
# --gpus 8 on a 1-GPU box.  Every GPU step has its own time limit; the first failure ends the call.
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
O=gpurun_out/r03
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 ${T:-900} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYARGS:-} > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --dtype fp16 --no-cpu-baseline > $O/bench_fp16.json 2> $O/bench_fp16.err
rc=$?; echo "bench fp16 rc=$rc"; cut -c1-400 $O/bench_fp16.json; [ $rc -eq 0 ] || { tail -20 $O/bench_fp16.err; exit $rc; }
SPMCTS_DIST_BACKEND=gloo SPMCTS_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 8 --warmup 3 \
  --no-cpu-baseline > $O/reh2.json 2> $O/reh2.err
rc=$?; echo "rehearsal rc=$rc"; cut -c1-300 $O/reh2.json; python -c "import json; d=json.load(open('$O/reh2.json')); print('n_gpus', d['n_gpus'], 'exchange', d['exchange'])"
[ $rc -eq 0 ] || { tail -20 $O/reh2.err; exit $rc; }
timeout -k 10 120 python -u bench.py --gpus 8 --steps 2 --warmup 1 > $O/refuse8.json 2> $O/refuse8.err
echo "gpus 8 on this box rc=$? (expected 2)"; cat $O/refuse8.err | tail -2
exit 0
