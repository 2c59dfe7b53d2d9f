# Round 5, trainer convolutions second form: GPU tests, trainer-only graphed step HIP vs MIOpen alternated,
# kernel trace of the HIP-conv step.
set -u
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainconv.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -100; exit $rc; }
timeout -k 10 600 python3 -u scripts/bench_train.py --conv-ab > $O/conv_ab.json 2> $O/conv_ab.err || { tail -5 $O/conv_ab.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/conv_ab.json').read().strip().splitlines()[-1]); print([(r['train_hip_convs'], round(r['ms_per_sgd_step'],2)) for r in d['trainer_only']])" | tee -a $O/summary.txt
bash scripts/gpu_r05e.sh | tee -a $O/summary.txt
exit 0
