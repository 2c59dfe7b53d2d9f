# Round 6, final tree: BASELINE configs[4] (arena evaluation, 8,192 games per GPU, two ResNet-128x20 nets, fp16,
# evaluate mode) in steady state (45 warm-up plies, 40 timed), configs[2] in steady state (one game generation of
# warm-up, 6 timed plies, 4 no-dedup twin plies; cross-lane dedup on), and the driver's bench command.
set -u
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --mode arena --games 8192 --warmup 45 --steps 40 --no-cpu-baseline \
  > $O/config5_arena_steady.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/config5_arena_steady.json') if l.startswith('{')][0]); print('config5', round(d['value'],1), d['unit'], round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], d['dtype'], d['roofline']['clock'].get('clock_ghz'))" | tee -a $O/summary.txt
T=900 bash scripts/gpu_config3_steady.sh && cp gpurun_out/cfg3/config3_steady_dedup.* $O/ || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/config3_steady_dedup.json') if l.startswith('{')][0]); print('config3', round(d['value'],1), round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], d['config']['cross_lane_dedup'], d['roofline']['clock'].get('clock_ghz'), (d.get('no_dedup_twin') or {}).get('value'))" | tee -a $O/summary.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_driver.json') if l.startswith('{')][0]); r=d['roofline']; print('driver', round(d['value']), 'frac', round(r['frac'],4), 'executed', round(r['executed']['frac'],4), 'clock', r['clock'].get('clock_ghz'), 'at_clock', r['clock'].get('frac_at_clock'), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'twin', d.get('no_dedup_twin', {}).get('value'))" | tee -a $O/summary.txt
exit 0
