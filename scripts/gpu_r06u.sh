# Round 6: k_scan_need before the evaluation cache (ab_libs/libspmcts_precache.so: commit e239688's spmcts.hip with
# this tree's tower / trainconv objects) vs now, both with the cache off (--eval-cache 0), kernel stats of the
# driver's command, one box.
set -u
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --twin-no-dedup 0 --twin-no-cache 0 --eval-cache 0"
for lib in precache now; do
  if [ $lib = precache ]; then export SPMCTS_LIB=$PWD/ab_libs/libspmcts_precache.so; else unset SPMCTS_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/t_$lib -o run -- python3 bench.py $ARGS > $O/$lib.json 2> $O/$lib.err
  rc=$?; echo "$lib rc=$rc" | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -5 $O/$lib.err; exit $rc; }
  cp $O/t_$lib/run_kernel_stats.csv $O/kernel_stats_$lib.csv && rm -f $O/t_$lib/run_kernel_trace.csv
  python3 -c "
import csv; rows=list(csv.DictReader(open('$O/kernel_stats_$lib.csv')))
print('$lib', [(r['Name'][:22], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'scan' in r['Name'] or 'owner' in r['Name'] or 'expand_vl' in r['Name']])" | tee -a $O/summary.txt
done
exit 0
