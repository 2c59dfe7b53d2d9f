# Round 6, last pass over the final tree: the whole -m gpu suite as the driver runs it (incl. the broadened
# cross-lane dedup cases and the 0.48 lane split), smoke(), the driver bench, then the multi-rank rehearsal.
set -u
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -s > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -120; exit $rc; }
grep -E "evaluate mode|config3|excess|rows/leaf" $O/tests.log | tee -a $O/summary.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log | tee -a $O/summary.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][0]); r=d['roofline']; print(round(d['value']), 'frac', round(r['frac'],4), 'executed', round(r['executed']['frac'],4), 'clock', r['clock'].get('clock_ghz'), 'at_clock', r['clock'].get('frac_at_clock'), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'cpu', d['cpu_baseline']['value'])" | tee -a $O/summary.txt
bash scripts/gpu_multirank_final.sh 2>&1 | tee -a $O/summary.txt
