"""The vendor GEMM's rate on the same box as the fused trunk, each with the clock of its own timed region.

What a 0.64 dense frac means on this chip: hipBLASLt (torch.matmul, fp16 in, fp32 accumulate) on
  * a large square GEMM (M = N = K = 8192),
  * the trunk's conv layer as one GEMM (im2col rows of 6,144 boards x 42 cells, K = 9 x 128, N = 128;
    im2col itself not timed, so this is a lower bound on a library conv layer's time),
timed with HIP events beside the fused trunk (6,144 boards, fp16, `HipTowerEvaluator.trunk`), alternated
`--reps` times; amdsmi's gfx clock is sampled over each timed region (bench.GfxClock).  Prints one JSON line.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench import GfxClock, head_linear_flops, resnet_flops_per_leaf
from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
from self_play_reinforcement_learning_amd.modules import ResidualTower, planes_from_boards

PEAK = 2.5e15  # dense fp16 / bf16 MFMA, MI355X_MICROARCH.md

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--batch", type=int, default=6144)
args = ap.parse_args()
dev = torch.device("cuda:0")


def timed(fn, flops, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    clk = GfxClock(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    clk.start()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    clk.stop()
    ms = e0.elapsed_time(e1) / iters
    c = clk.report().get("clock_ghz")
    rate = flops / (ms * 1e-3)
    return {"us": round(ms * 1e3, 1), "tflops": round(rate / 1e12, 1), "frac": round(rate / PEAK, 4),
            "clock_ghz": round(c, 3) if c else None,
            "frac_at_clock": round(rate / (PEAK * c / 2.4), 4) if c else None}


torch.manual_seed(0)
a = torch.randn(8192, 8192, device=dev, dtype=torch.float16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.float16)
rows = args.batch * 42
ai = torch.randn(rows, 9 * 128, device=dev, dtype=torch.float16)
wi = torch.randn(9 * 128, 128, device=dev, dtype=torch.float16)
net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32).to(dev).eval()
x = planes_from_boards(torch.randint(-1, 2, (args.batch, 7, 6)), 7, 6).to(dev).to(torch.bfloat16)
xt = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
ev = HipTowerEvaluator(net, dtype=torch.float16)
trunk_flops = (resnet_flops_per_leaf(7, 6, 7, 32, 20) - head_linear_flops(7, 6, 7, 32)) * args.batch  # 496.43 MFLOP/board
cases = {
    "hipblaslt_8192_cubed": (lambda: torch.matmul(a, b), 2 * 8192 ** 3),
    "hipblaslt_trunk_layer_gemm": (lambda: torch.matmul(ai, wi), 2 * rows * 9 * 128 * 128),
    "fused_trunk_fp16": (lambda: ev.trunk(xt), trunk_flops),
}
out = {"batch": args.batch, "iters": args.iters, "peak_tflops": PEAK / 1e12,
       "note": "fused_trunk flops are the dense-equivalent (bench.resnet_flops_per_leaf); its executed MFMA work is 5/6 of "
               "the residual blocks' dense FLOPs", "runs": {k: [] for k in cases}}
for _ in range(args.reps):
    for k, (fn, fl) in cases.items():
        out["runs"][k].append(timed(fn, fl, args.iters))
print(json.dumps(out))
