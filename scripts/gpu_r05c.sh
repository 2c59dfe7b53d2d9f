# Round 5: BASELINE configs[4] (arena evaluation, 8,192 games per GPU, two ResNet-128x20 nets, 200 sims, fp16
# trunk, evaluate mode) in steady state (45 warm-up plies, 40 timed), then configs[2] in steady state
# (scripts/gpu_config3_steady.sh: one game generation of warm-up, 6 timed plies, 4 no-dedup twin plies).
set -u
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --mode arena --games 8192 --warmup 45 --steps 40 --no-cpu-baseline \
  > $O/config5_arena_steady.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/config5_arena_steady.json') if l.startswith('{')][0]); print('config5', round(d['value'],1), d['unit'], round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], d['dtype'])" | tee -a $O/summary.txt
T=900 bash scripts/gpu_config3_steady.sh && cp gpurun_out/cfg3/config3_steady_dedup.* $O/ 2>/dev/null
exit 0
