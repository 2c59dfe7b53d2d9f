# Round 6, final tree (shared lane cache): BASELINE configs[4] (arena evaluation, 8,192 games per GPU, two
# ResNet-128x20 nets, fp16, evaluate mode, evaluation cache window 1) in steady state (45 warm-up plies, 40 timed),
# with its no-cache twin, then the profile bundle of the driver's command (scripts/gpu_r06l.sh).
set -u
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python3 -u bench.py --mode arena --games 8192 --warmup 45 --steps 40 --no-cpu-baseline --twin-no-cache 8 \
  --twin-no-dedup 0 > $O/config5_arena_steady_cache.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/config5_arena_steady_cache.json') if l.startswith('{')][0]); t=d.get('no_cache_twin') or {}; print('config5', round(d['value'],1), d['unit'], round(d['roofline']['frac'],4), round(d['nn']['rows_per_leaf'],4), d['nn']['cache_rows'], d['dtype'], d['roofline']['clock'].get('clock_ghz'), 'no-cache twin', t.get('value'), t.get('rows_per_leaf'))" | tee -a $O/summary.txt
bash scripts/gpu_r06l.sh
