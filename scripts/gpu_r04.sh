# Round 4 verification pass on the current tree: the whole -m gpu suite, smoke, the driver-form bench
# (python bench.py --steps 20 --warmup 5: fp16 headline + no-dedup twin + bf16 secondary + cpu_baseline),
# then the trainer throughput (scripts/bench_train.py: graphed vs eager SGD steps, self-play beside them).
# STAGES: subset of "tests bench train" (default all).  Own time limit per step; stops at the first failure.
set -u
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
ST=${STAGES:-tests bench train}
if [[ " $ST " == *" tests "* ]]; then
  timeout -k 10 ${T:-1000} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/gpu_tests.log | head -100; exit $rc; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [[ " $ST " == *" bench "* ]]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
sec = d.get('secondary_dtype')
print('bench', d['dtype'], round(d['value']), round(d['roofline']['frac'],4), 'twin', round(d['no_dedup_twin']['value']),
      'secondary', (sec['dtype'], round(sec['value']), round(sec['roofline']['frac'],4)) if sec else None,
      'cpu', round(d['cpu_baseline']['value'],2))"
fi
if [[ " $ST " == *" train "* ]]; then
  timeout -k 10 600 python -u scripts/bench_train.py --plies ${TPLIES:-16} > $O/train.json 2> $O/train.err || { tail -5 $O/train.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/train.json').read().strip().splitlines()[-1])
for r in d['trainer_only']: print('trainer-only', r['train_graph'], r['train_autocast'], round(r['ms_per_sgd_step'],2), 'ms/step')
for r in d['runs']: print('selfplay+train', r['updates_per_ply'], 'graph', r['train_graph'], 'stream', r['trainer_stream'], round(r['positions_per_s']), 'pos/s', round(r['sgd_steps_per_s'],1), 'steps/s')"
fi
exit 0
