# Round 6: lane 0's stream at high priority (SPMCTS_LANE_PRIORITY=1, engine.py) with the evaluation cache's shorter
# towers, the driver's form alternated twice on one box.
set -u
O=gpurun_out/r06y
mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']
print(sys.argv[2], round(d['value']), 'ms/ply', round(d['ms_per_step'],2), 'frac', round(r['frac'],4), 'clock', round(r['clock'].get('clock_ghz') or 0,3), 'nn_share', round(d['nn']['share_of_step'],4))" "$1" "$2"; }
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0"
for rep in 1 2; do
  for p in 0 1; do
    SPMCTS_LANE_PRIORITY=$p timeout -k 10 300 python3 bench.py $ARGS > $O/prio${p}_$rep.json 2> $O/prio${p}_$rep.err || { tail -20 $O/prio${p}_$rep.err; exit 1; }
    line $O/prio${p}_$rep.json "lane priority $p rep $rep:" | tee -a $O/summary.txt
  done
done
exit 0
