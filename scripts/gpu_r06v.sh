# Round 6: the bench-line GPU tests after the twin-unit change, then the driver's exact command once more.
set -u
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "bench_line or bench_arena" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][0]); r=d['roofline']; print('driver', round(d['value']), 'frac', round(r['frac'],4), 'executed', round(r['executed']['frac'],4), 'clock', r['clock'].get('clock_ghz'), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'rows/launch', round(r['rows_per_launch']), 'no-cache twin', round(d['no_cache_twin']['value']), 'no-dedup twin', round(d['no_dedup_twin']['value']), 'cpu', d['cpu_baseline']['value'])" | tee -a $O/summary.txt
exit 0
