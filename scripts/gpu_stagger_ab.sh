# Staggered lanes (engine.LanedEngine stagger, bench.py --stagger) against lanes in lock step (the default):
# (1) the engine GPU tests (laned engine == its lanes, bench end to end); (2) a steady-state kernel trace
# of the bench (42 warm-up plies, 7 traced) with its tower-free windows by ply phase, staggered;
# (3) the driver-form bench (warm-up 5, 20 plies) and a steady-state run (warm-up 42, 12 plies),
# staggered vs lock step, alternated on one box.
set -u
O=gpurun_out/stagger
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/engine_tests.log 2>&1
rc=$?; tail -2 $O/engine_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/engine_tests.log | head -80; exit $rc; }
fi
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- \
  python3 bench.py --warmup 42 --steps 7 --no-cpu-baseline --twin-no-dedup 0 --no-secondary --stagger > $O/bench_traced.json 2> $O/trace.err
rc=$?; echo "steady trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 scripts/trace_idle.py $O/trace/run_kernel_trace.csv 7 2 > $O/trace_idle.json && cat $O/trace_idle.json
gzip -f $O/trace/run_kernel_trace.csv
val() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), d['config'].get('lanes_staggered'))" "$1"; }
for rep in 1 2; do
  for v in stagger lockstep; do
    if [ $v = stagger ]; then F="--stagger"; else F=""; fi
    timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 --no-secondary $F > $O/short_$v.json 2> $O/short_$v.err || { tail -5 $O/short_$v.err; exit 1; }
    echo "short $v: $(val $O/short_$v.json)" | tee -a $O/summary.txt
    timeout -k 10 300 python3 bench.py --warmup 42 --steps 12 --no-cpu-baseline --twin-no-dedup 0 --no-secondary $F > $O/steady_$v.json 2> $O/steady_$v.err || { tail -5 $O/steady_$v.err; exit 1; }
    echo "steady $v: $(val $O/steady_$v.json)" | tee -a $O/summary.txt
  done
done
exit 0
