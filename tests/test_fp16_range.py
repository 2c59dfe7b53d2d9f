"""CPU: the fp16 fused tower cannot overflow on the bench's nets.

The fp16 trunk (csrc/tower.hip, SPMCTS_TOWER_F16) keeps every layer's output in fp16 between layers,
as the reference's own inference does under fp16 autocast (inference_worker.py:117).  fp16's largest
finite value is 65504.  Here the bench's networks as bench.py builds them (ResidualTower(7, 6, 7,
num_blocks=20, filter_factor=32 / 64), torch.manual_seed(0), BatchNorm at init statistics; configs 2
and 3) run in fp32 on random boards, and every conv / BatchNorm / residual-block output must stay
below 65504 / 64 = 1023.5 in magnitude: a 64x headroom (measured maximum about 10).
"""
import numpy as np
import pytest
import torch

from self_play_reinforcement_learning_amd.modules import ResidualTower, planes_from_boards

FP16_MAX = 65504.0


@pytest.mark.parametrize("ff", [32, 64])
def test_bench_net_activations_far_inside_fp16_range(ff):
    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=ff).eval()
    peak = {}

    def hook(name):
        def f(_m, _i, o):
            peak[name] = max(peak.get(name, 0.0), float(o.detach().abs().max()))
        return f

    blocks = set(id(b) for b in net.residual_blocks)
    for name, m in net.named_modules():
        if isinstance(m, (torch.nn.Conv2d, torch.nn.BatchNorm2d, torch.nn.Linear)) or id(m) in blocks:
            m.register_forward_hook(hook(name))
    rng = np.random.default_rng(0)
    boards = rng.choice([-1, 0, 1], size=(48, 7, 6), p=[0.3, 0.4, 0.3])
    boards[0] = 0  # the empty board (every search's root)
    with torch.no_grad():
        net.forward_planes(planes_from_boards(torch.as_tensor(boards), 7, 6))
    assert len(peak) >= 4 * 20
    worst = max(peak.values())
    assert worst < FP16_MAX / 64, sorted(peak.items(), key=lambda kv: -kv[1])[:3]
