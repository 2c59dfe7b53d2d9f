# Round 6: the evaluation cache shared by paired lanes (a follower uses its leader's table).  The cache and dedup
# exactness tests, then the driver's command: shared vs per-lane tables (A/B library, SPMCTS_CACHE_SHARE=0 is the
# per-lane form) alternated twice, then the product library at lane splits 0.44 / 0.48 / 0.52.
set -u
O=gpurun_out/r06n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "eval_cache or dedup" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|rows/leaf" $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],1), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'cache_rows', d['nn']['cache_rows'], 'lanes', d['config']['lane_games'])" "$1" "$2"; }
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
for rep in 1 2; do
  for sh in 1 0; do
    SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so SPMCTS_CACHE_SHARE=$sh timeout -k 10 300 \
      python3 bench.py $ARGS > $O/share${sh}_$rep.json 2> $O/share${sh}_$rep.err || { tail -20 $O/share${sh}_$rep.err; exit 1; }
    line $O/share${sh}_$rep.json "ab share=$sh rep $rep:" | tee -a $O/summary.txt
  done
done
for s in 0.44 0.48 0.52; do
  timeout -k 10 300 python3 bench.py $ARGS --lane0-share $s > $O/split_$s.json 2> $O/split_$s.err || { tail -20 $O/split_$s.err; exit 1; }
  line $O/split_$s.json "product split $s:" | tee -a $O/summary.txt
done
exit 0
