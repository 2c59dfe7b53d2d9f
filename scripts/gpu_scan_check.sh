# k_scan_need as a two-level shuffle scan: the parity / engine GPU tests (row assignment is what every
# leaf's evaluation reads), then a kernel trace of the bench (kernel stats: k_scan_need's mean duration,
# 37.4 us in profiles/r04_bench_prof/kernel_stats.csv before the change).
set -u
O=gpurun_out/scan
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | head -60; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 bench.py --steps 3 --warmup 24 --no-cpu-baseline --twin-no-dedup 0 > $O/bench_traced.json 2> $O/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_scan_need', 'k_expand_vl', 'k_heads_co', 'k_dedup', 'k_encode', 'k_select_vl')):
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
"
