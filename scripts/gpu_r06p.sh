# Round 6: lanes per GPU with the shared evaluation cache (2 = the default, 3 = two followers on lane 0's table),
# the driver's form, alternated twice on one box.
set -u
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],1), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'rows/leaf', round(d['nn']['rows_per_leaf'],4), 'nn_share', round(d['nn']['share_of_step'],4), 'lanes', d['config']['lane_games'])" "$1" "$2"; }
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
for rep in 1 2; do
  for l in 2 3; do
    timeout -k 10 300 python3 bench.py $ARGS --lanes $l > $O/lanes${l}_$rep.json 2> $O/lanes${l}_$rep.err || { tail -20 $O/lanes${l}_$rep.err; exit 1; }
    line $O/lanes${l}_$rep.json "lanes $l rep $rep:" | tee -a $O/summary.txt
  done
done
exit 0
