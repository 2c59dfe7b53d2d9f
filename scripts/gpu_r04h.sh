# (1) the engine / parity GPU tests (k_scan_need at 512 threads among them); (2) the driver-form bench
# twice; (3) a kernel trace of the bench (k_scan_need beside the trunk).
# (Commit 24bacd3's version of this script also timed the GEMM-form trainer convolutions,
# profiles/r04/trainer/gemm_rows_ab.json; that path was measured slower and removed.)
set -u
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | head -60; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > $O/b$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  echo "bench: $(python3 -c "import json; d=json.loads([l for l in open('$O/b$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['no_dedup_twin']['value']))")"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 24 --no-cpu-baseline --twin-no-dedup 0 > $O/traced.json 2> $O/trace.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
rm -f $O/trace/run_kernel_trace.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/trace/run_kernel_stats.csv')))[:6]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'][:5], round(float(r['MinNs'])/1e3,1))"
exit 0
