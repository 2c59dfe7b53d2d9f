"""Micro-benchmark: fused HIP tower vs PyTorch bf16 path for the leaf evaluator (ResNet-128x20, 4096 boards)."""
import argparse
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench import resnet_flops_per_leaf
from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator, TowerEvaluator
from self_play_reinforcement_learning_amd.modules import ResidualTower, planes_from_boards

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--ff", type=int, default=32)
ap.add_argument("--blocks", type=int, default=20)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--trunk-only", action="store_true")
ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16", help="the fused trunk's element type")
args = ap.parse_args()
torch.manual_seed(0)
net = ResidualTower(7, 6, 7, num_blocks=args.blocks, filter_factor=args.ff).cuda().eval()
b = torch.randint(-1, 2, (args.batch, 7, 6))
x = planes_from_boards(b, 7, 6).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
fl = resnet_flops_per_leaf(7, 6, 7, args.ff, args.blocks) * args.batch
out = {}
if args.trunk_only:
    ev = HipTowerEvaluator(net, dtype={"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype])
    xt = x.permute(0, 2, 3, 1)
    for _ in range(3):
        ev.trunk(xt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        ev.trunk(xt)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps(dict(batch=args.batch, dtype=args.dtype, cg=os.environ.get("SPMCTS_TOWER_CG"), trunk_ms=ms,
                          tflops=fl / ms / 1e9)))
    sys.exit(0)
for name, ev in (("hip", HipTowerEvaluator(net)), ("hip_fusedheads", HipTowerEvaluator(net, fused_heads=True)),
                 ("hip_torchheads", HipTowerEvaluator(net, fused_heads=False)),
                 ("torch_bf16", TowerEvaluator(net, dtype=torch.bfloat16))):
    for _ in range(3):
        ev(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        ev(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    out[name] = dict(ms=ms, tflops=fl / ms / 1e9)
    if name == "hip":
        e0.record()
        for _ in range(args.iters):
            ev.trunk(x.permute(0, 2, 3, 1))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        out["hip_trunk_only"] = dict(ms=ms, tflops=fl / ms / 1e9)
print(json.dumps(dict(batch=args.batch, ff=args.ff, blocks=args.blocks, **out)))
