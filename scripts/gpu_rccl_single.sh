# RCCL (backend "nccl") rehearsal on a 1-GPU box: RCCL refuses two ranks on one device, so the
# multi-GPU code path runs as ONE rank with a real process group (SPMCTS_DIST_SINGLE=1): every
# collective the driver's N-GPU bench issues — the header all_gather and the row gather of each
# MoveExchange round, the max-over-ranks all_reduce, barrier(device_ids=...), init_process_group(
# device_id=...) — and the scheduler's one-buffer weight broadcast, on RCCL with device tensors.
set -u
O=gpurun_out/rccl1
mkdir -p $O
export TMPDIR=/tmp SPMCTS_DIST_BACKEND=nccl SPMCTS_DIST_SINGLE=1 NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29573 bench.py --gpus 1 --steps 16 --warmup 8 --games 2048 --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err
rc=$?; echo "rccl single-rank bench rc=$rc"; [ $rc -eq 0 ] || { tail -25 $O/bench.err; exit $rc; }
python -c "import json; d=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0]); print(round(d['value']), d['n_gpus'], json.dumps(d.get('exchange')))"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29574 scripts/rehearse_multirank.py > $O/scheduler.json 2> $O/scheduler.err
rc=$?; echo "rccl single-rank scheduler rc=$rc"; cat $O/scheduler.json; [ $rc -eq 0 ] || { tail -25 $O/scheduler.err; exit $rc; }
grep -i "nccl\|rccl" $O/bench.err | head -5
exit 0
