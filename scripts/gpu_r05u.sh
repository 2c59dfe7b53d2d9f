# Round 5: config 3 in steady state (one game generation of warm-up: 42 plies, 6 timed) with the C = 256
# trunk on 16x16x32 one-buffer tiles (tower_wide16.h) and the round's tree kernels.
set -u
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1080 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 42 --steps 6 \
  --blocks-per-tree 8000 --twin-no-dedup 0 --no-cpu-baseline --progress > $O/c3_steady.json 2> $O/c3_steady.err || { tail -3 $O/c3_steady.err; exit 1; }
echo "config3 steady: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_steady.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], round(d['nn']['share_of_step'],4), round(d['ms_per_step'],1))")" | tee -a $O/summary.txt
exit 0
