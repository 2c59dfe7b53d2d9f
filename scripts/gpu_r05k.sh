# Round 5: config 3 (16,384 games, 800 sims, ResNet-256x20) near steady state (32 warm-up plies, 6 timed), two lanes
# vs three lanes per GPU, same box.
set -u
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
for lanes in 3 2; do
  timeout -k 10 540 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 32 --steps 6 \
    --blocks-per-tree 8000 --twin-no-dedup 0 --no-cpu-baseline --progress --lanes $lanes \
    > $O/c3_lanes$lanes.json 2> $O/c3_lanes$lanes.err || { tail -3 $O/c3_lanes$lanes.err; exit 1; }
  echo "config3 lanes $lanes: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_lanes$lanes.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
done
exit 0
