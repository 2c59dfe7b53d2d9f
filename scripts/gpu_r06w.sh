# Round 6: one host round trip per ply boundary (every lane's finish + Move export queued into persistent buffers
# before the host waits) vs the previous engine (ab_py/: the package and bench.py of the commit before, on this
# tree's library), the driver's form alternated twice; the parity and engine GPU tests first.
set -u
O=gpurun_out/r06w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 600 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/tests.log | head -120; exit $rc; }
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],2), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'nn_share', round(d['nn']['share_of_step'],4))" "$1" "$2"; }
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
for rep in 1 2; do
  SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/libspmcts.so timeout -k 10 300 python3 ab_py/bench.py $ARGS \
    > $O/prev_$rep.json 2> $O/prev_$rep.err || { tail -20 $O/prev_$rep.err; exit 1; }
  line $O/prev_$rep.json "previous engine rep $rep:" | tee -a $O/summary.txt
  timeout -k 10 300 python3 bench.py $ARGS > $O/new_$rep.json 2> $O/new_$rep.err || { tail -20 $O/new_$rep.err; exit 1; }
  line $O/new_$rep.json "one round trip rep $rep:" | tee -a $O/summary.txt
done
exit 0
