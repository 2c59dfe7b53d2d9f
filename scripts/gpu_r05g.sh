# Round 5: isolated tree kernels on steady-state trees (24 warm-up plies, table net, 4,096 games, K = 4) with
# the worst-case node store (no recycling) and with recycled stores of 1,400 / 2,000 blocks per tree: does the
# store's footprint (TLB / Infinity-Cache reach) set the steady-state select / expand times?
set -u
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
for bpt in 0 1400 2000 0 1400; do
  timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 --blocks-per-tree $bpt > $O/iso_$bpt.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  echo "bpt $bpt: $(python3 -c "import json; d=json.loads(open('$O/iso_$bpt.json').read().strip().splitlines()[-1]); print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k in ('select_avg_us', 'expand_avg_us', 'ply_ms', 'mean_levels', 'compactions', 'blocks_in_use_max', 'blocks_per_tree')})")" | tee -a $O/summary.txt
done
exit 0
