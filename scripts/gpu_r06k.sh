# Round 6: the evaluation cache (include/spmcts.h spmcts_set_eval_cache).  First its exactness tests and the
# dedup tests beside them, then the driver's command with the cache window 0 / 1 / 2, alternated on one box.
set -u
O=gpurun_out/r06k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "eval_cache or dedup" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|rows/leaf" $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
for rep in 1 2; do
  for w in 0 1 2; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --eval-cache $w \
      > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err || { tail -20 $O/bench_w${w}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/bench_w${w}_$rep.json') if l.startswith('{')][0]); r=d['roofline']; t=d.get('no_cache_twin') or {}
print('window $w rep $rep:', round(d['value']), 'ms/ply', round(d['ms_per_step'],1), 'frac', round(r['frac'],4), 'clock', r['clock'].get('clock_ghz'), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'cache_rows', d['nn']['cache_rows'], 'nn_share', round(d['nn']['share_of_step'],3), 'twin', round(t.get('value',0)), round(t.get('rows_per_leaf',0),4))" | tee -a $O/summary.txt
  done
done
exit 0
