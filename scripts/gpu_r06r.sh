# Round 6, final tree: (1) the driver's workload in steady state (45 warm-up plies: every game slot has been refilled
# at least once) with the evaluation cache (window 1) vs without (--eval-cache 0), alternated; (2) configs[2] in
# steady state with the shared-table cache (scripts/gpu_config3_steady.sh).
set -u
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],1), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'cache_rows', d['nn']['cache_rows'], 'nn_share', round(d['nn']['share_of_step'],4))" "$1" "$2"; }
ARGS="--gpus 1 --steps 12 --warmup 45 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0 --progress"
for w in 1 0; do
  timeout -k 10 300 python3 bench.py $ARGS --eval-cache $w > $O/steady_w$w.json 2> $O/steady_w$w.err || { tail -20 $O/steady_w$w.err; exit 1; }
  line $O/steady_w$w.json "steady state, window $w:" | tee -a $O/summary.txt
done
T=1000 TAG=shared TWIN=0 EXTRA="--twin-no-cache 0" bash scripts/gpu_config3_steady.sh && cp gpurun_out/cfg3/config3_steady_shared.* $O/ || exit 1
line $O/config3_steady_shared.json "config3 steady, shared cache:" | tee -a $O/summary.txt
exit 0
