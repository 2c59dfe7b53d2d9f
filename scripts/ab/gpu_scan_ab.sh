# Leaf-row scan with per-slot owner flags (k_dedup_owner) and unrolled chunk loops: dedup/engine GPU
# tests, then the kernel stats of a short traced bench and the bench itself.
set -u
mkdir -p gpurun_out/scan
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -x -q -m gpu -k "dedup or threaded or full_size" --timeout 200 --timeout-method thread > gpurun_out/scan/tests.log 2>&1
rc=$?; tail -1 gpurun_out/scan/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/scan/tests.log | head -20; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/scan/trace -o run -- python3 bench.py --warmup 8 --steps 3 --no-cpu-baseline > gpurun_out/scan/traced.json 2> gpurun_out/scan/trace.err
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/scan/trace.err; exit $rc; fi
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/scan/trace/run_kernel_stats.csv')))[:8]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
