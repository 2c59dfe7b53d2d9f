# Multi-rank paths on the final tree, one 1-GPU box: bench.py's self-launch (`--gpus 2` without torchrun,
# SPMCTS_ALLOW_OVERSUBSCRIBE=1 + gloo: two rank processes on the one GPU), torchrun's 2-rank gloo form,
# and the RCCL one-rank group (scripts/gpu_rccl_single.sh).  Own time limit per step.
set -u
O=gpurun_out/multirank
mkdir -p $O
export TMPDIR=/tmp
SPMCTS_ALLOW_OVERSUBSCRIBE=1 SPMCTS_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 8 --warmup 3 \
  --games 2048 --no-cpu-baseline --twin-no-dedup 0 > $O/selflaunch.json 2> $O/selflaunch.err
rc=$?; echo "self-launch rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/selflaunch.err; exit $rc; }
python3 -c "import json; d=json.loads([l for l in open('$O/selflaunch.json') if l.startswith('{')][0]); print(round(d['value']), d['n_gpus'], d['exchange'], d.get('ranks'))"
SPMCTS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 8 --warmup 3 --games 2048 --no-cpu-baseline --twin-no-dedup 0 \
  > $O/torchrun.json 2> $O/torchrun.err
rc=$?; echo "torchrun rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/torchrun.err; exit $rc; }
python3 -c "import json; d=json.loads([l for l in open('$O/torchrun.json') if l.startswith('{')][0]); print(round(d['value']), d['n_gpus'], d['exchange'], d.get('ranks'))"
bash scripts/gpu_rccl_single.sh
