# Round 6, the rebuilt libraries of the final tree: the cache / dedup / bench-line GPU tests, smoke(), the driver's
# exact command.
set -u
O=gpurun_out/r06x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "eval_cache or dedup or bench_ or games or threaded" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | tee -a $O/summary.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][0]); r=d['roofline']; print('driver', round(d['value']), 'frac', round(r['frac'],4), 'clock', r['clock'].get('clock_ghz'), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'no-cache twin', round(d['no_cache_twin']['value']), 'no-dedup twin', round(d['no_dedup_twin']['value']))" | tee -a $O/summary.txt
exit 0
