# (1) the engine / parity GPU tests that exercise k_scan_need (256 threads) and the trainer (GEMM-form
# convolutions, graph vs eager exact under deterministic algorithms); (2) trainer-only ms per SGD step,
# GEMM-form vs the convolution library, graphed / eager, fp16 autocast / fp32; (3) the driver-form bench
# twice; (4) a kernel trace of the bench (k_scan_need beside the trunk).
set -u
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py::test_trainer_graph_train_mode_replays_run -m gpu -x -q --timeout 120 --timeout-method thread > $O/one.log 2>&1; echo "one rc=$?"; grep "AssertionError" $O/one.log | head -3
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py::test_trainer_graph_train_mode_replays_run -m gpu -x -q > $O/one2.log 2>&1; echo "one (no timeout plugin) rc=$?"; grep "AssertionError" $O/one2.log | head -3
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | head -60; exit $rc; }
timeout -k 10 400 python3 scripts/bench_train.py --trainer-gemm-ab > $O/train_ab.json 2> $O/train_ab.err || { tail -5 $O/train_ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/train_ab.json'))
for r in d['trainer_only']: print('trainer graph', r['train_graph'], 'autocast', r['train_autocast'], 'gemm', r['gemm_convs'], round(r['ms_per_sgd_step'],2), 'ms', round(r['last_loss'],4))"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > $O/b$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
  echo "bench: $(python3 -c "import json; d=json.loads([l for l in open('$O/b$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['no_dedup_twin']['value']))")"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 24 --no-cpu-baseline --twin-no-dedup 0 > $O/traced.json 2> $O/trace.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
rm -f $O/trace/run_kernel_trace.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/trace/run_kernel_stats.csv')))[:6]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'][:5])"
exit 0
