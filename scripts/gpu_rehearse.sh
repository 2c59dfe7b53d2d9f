# 2 ranks on the box's one GPU over gloo: bench.py and the scheduler rehearsal.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp SPMCTS_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
  bench.py --gpus 2 --steps 8 --warmup 3 --games ${GAMES:-4096} --no-cpu-baseline > gpurun_out/reh_bench.json 2> gpurun_out/reh_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/reh_bench.json | cut -c1-400; if [ $rc -ne 0 ]; then tail -20 gpurun_out/reh_bench.err; exit $rc; fi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 \
  scripts/rehearse_multirank.py > gpurun_out/reh_sched.out 2> gpurun_out/reh_sched.err
rc=$?; echo "sched rc=$rc"; grep rank gpurun_out/reh_sched.out; if [ $rc -ne 0 ]; then tail -20 gpurun_out/reh_sched.err; fi
exit $rc
