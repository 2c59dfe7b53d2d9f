# Round 6: BASELINE configs[2] (ResNet-256x20, 800 sims, 16,384 games) in steady state with the evaluation cache
# (bench.py's default window 1): one game generation of warm-up, 6 timed plies, then 3 plies with the cache off
# (no_cache_twin: per-step dedup alone) and 2 with dedup off (no_dedup_twin).
set -u
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
T=1080 TAG=cache TWIN=2 EXTRA="--twin-no-cache 3" bash scripts/gpu_config3_steady.sh && cp gpurun_out/cfg3/config3_steady_cache.* $O/ || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/config3_steady_cache.json') if l.startswith('{')][0]); print('config3', round(d['value'],1), round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], d['nn']['cache_rows'], d['roofline']['clock'].get('clock_ghz'), (d.get('no_cache_twin') or {}).get('value'), (d.get('no_cache_twin') or {}).get('rows_per_leaf'), (d.get('no_dedup_twin') or {}).get('value'))" | tee -a $O/summary.txt
exit 0
