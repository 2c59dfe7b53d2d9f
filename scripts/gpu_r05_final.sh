# Round-5 final-tree GPU pass, one box: the -m gpu tests (SKIP_STAT=1: without the statistical file;
# ONLY_STAT=1: that file alone, then stop), smoke(), then the driver's bench command
# (python bench.py --gpus 1 --steps 20 --warmup 5).
set -u
O=gpurun_out/r05_final
mkdir -p $O
export TMPDIR=/tmp
TARGETS="tests"
TAG=all
if [ -n "${ONLY_STAT:-}" ]; then TARGETS="tests/test_gpu_statistical.py"; TAG=stat;
elif [ -n "${SKIP_STAT:-}" ]; then TARGETS="tests --ignore=tests/test_gpu_statistical.py"; TAG=nostat; fi
timeout -k 10 1000 python -u -m pytest $TARGETS -m gpu -q -s --timeout 600 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 $O/gpu_tests_$TAG.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/gpu_tests_$TAG.log | head -120; exit $rc; }
[ -n "${ONLY_STAT:-}" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0]); print('bench', round(d['value']), d['dtype'], round(d['roofline']['frac'],4), round(d['ms_per_step'],1), d['no_dedup_twin']['value'] if d.get('no_dedup_twin') else None, d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)" | tee -a $O/summary.txt
exit 0
