# The bench's multi-rank path on RCCL (backend "nccl") with 2 ranks sharing the box's one GPU, short
# and under its own time limit: checks the exchange rounds, barrier and max-over-ranks timing on the
# collective library the driver's 8-GPU run uses.  Measured: RCCL refuses two ranks on one device
# ("Duplicate GPU detected", profiles/r02/rccl_2rank_one_gpu.txt); kept for multi-GPU boxes.
set -u
mkdir -p gpurun_out/nccl
export TMPDIR=/tmp SPMCTS_DIST_BACKEND=nccl NCCL_DEBUG=WARN
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 \
  bench.py --gpus 2 --steps 8 --warmup 3 --games ${GAMES:-1024} --no-cpu-baseline > gpurun_out/nccl/bench.json 2> gpurun_out/nccl/bench.err
rc=$?; echo "nccl bench rc=$rc"; cut -c1-400 gpurun_out/nccl/bench.json; [ $rc -eq 0 ] || tail -25 gpurun_out/nccl/bench.err
exit $rc
