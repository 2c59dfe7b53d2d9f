# Round 5: the trainer's 3x3 block convolutions on the HIP matrix-core kernels (trainconv.hip): GPU tests
# (vs torch fp32 convolution, trainer step vs MIOpen, graphed determinism, G8 on the GPU), then the
# trainer-only graphed step HIP vs MIOpen alternated, a kernel trace of the HIP-conv step, and the
# self-play + training throughput.
set -u
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainconv.py tests/test_trainer_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -100; exit $rc; }
timeout -k 10 600 python3 -u scripts/bench_train.py --conv-ab > $O/conv_ab.json 2> $O/conv_ab.err || { tail -5 $O/conv_ab.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/conv_ab.json').read().strip().splitlines()[-1]); print([(r['train_hip_convs'], round(r['ms_per_sgd_step'],2)) for r in d['trainer_only']])" | tee -a $O/summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/r05d_prof -o run -- python3 scripts/bench_train.py --trainer-only-graph > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
find /tmp/r05d_prof -name "*kernel_stats.csv" -exec cp {} $O/trainer_step_kernel_stats.csv \;
rm -rf /tmp/r05d_prof
timeout -k 10 900 python3 -u scripts/bench_train.py --plies 24 --updates 4 > $O/train_throughput.json 2> $O/tt.err || { tail -5 $O/tt.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/train_throughput.json').read().strip().splitlines()[-1]); print([(r['train_hip_convs'], round(r['ms_per_sgd_step'],2)) for r in d['trainer_only']]); print([(r['updates_per_ply'], r['train_hip_convs'], r['trainer_stream'], round(r['positions_per_s'])) for r in d['runs']])" | tee -a $O/summary.txt
exit 0
