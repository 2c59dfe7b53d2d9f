"""Where a NaN enters the GEMM-form (channels-last rows) trainer step in train mode under fp16 autocast:
losses of eager steps, then one step under autograd anomaly detection, and per-layer forward checks."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from self_play_reinforcement_learning_amd.mcts import az_loss
from self_play_reinforcement_learning_amd.modules import ResidualTower, _bn_rows, _conv3x3_rows, planes_from_boards

torch.manual_seed(0)
g = torch.Generator().manual_seed(1)
s = torch.randint(-1, 2, (64, 7, 6), generator=g)
pi = torch.full((64, 7), 1 / 7)
z = torch.randint(-1, 2, (64,), generator=g).float()
q = torch.zeros(64, dtype=torch.float64)
for autocast in (False, True):
    for rows in (False, True):
        torch.manual_seed(0)
        net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=16).cuda()
        net.gemm_convs = rows
        opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
        losses = []
        for i in range(4):
            net.train()
            with torch.autocast("cuda", dtype=torch.float16, enabled=autocast):
                loss = az_loss(net, s.cuda(), z.cuda(), pi.cuda(), q.cuda(), True)
                opt.zero_grad()
                loss.backward()
                bad = [n for n, p in net.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
                opt.step()
            losses.append(round(float(loss), 5))
            if bad:
                losses.append(("nonfinite grads", bad[:6]))
        print("autocast", autocast, "rows", rows, losses, flush=True)
# forward of the rows path, layer by layer, in train mode under autocast
torch.manual_seed(0)
net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=16).cuda().train()
x = planes_from_boards(s, 7, 6).cuda()
with torch.autocast("cuda", dtype=torch.float16):
    r = x.permute(0, 2, 3, 1)
    c = _conv3x3_rows(r, net.conv1)
    print("stem conv", c.dtype, bool(torch.isfinite(c).all()), float(c.float().abs().max()))
    b = _bn_rows(net.bn1, c)
    print("stem bn", b.dtype, bool(torch.isfinite(b).all()), float(b.float().abs().max()),
          "running_var finite", bool(torch.isfinite(net.bn1.running_var).all()))
    ref = torch.nn.functional.batch_norm(c.float().reshape(-1, c.shape[-1]), None, None, net.bn1.weight, net.bn1.bias, True,
                                         0.1, 1e-5)
    print("stem bn vs fp32", float((b.float().reshape(ref.shape) - ref).abs().max()))
with torch.autograd.detect_anomaly():
    net.gemm_convs = True
    with torch.autocast("cuda", dtype=torch.float16):
        loss = az_loss(net, s.cuda(), z.cuda(), pi.cuda(), q.cuda(), True)
    print("anomaly-mode loss", float(loss), flush=True)
    try:
        loss.backward()
        print("backward ok")
    except RuntimeError as e:
        print("anomaly:", str(e)[:400])
