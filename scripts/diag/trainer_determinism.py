"""Run-to-run spread of the trainer's weights after 10 SGD steps (ResNet 2 blocks, batch 64): eager twice,
graphed twice, in fp32 and under fp16 autocast, printing each tensor group's relative update difference."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from self_play_reinforcement_learning_amd.modules import ResidualTower  # noqa: E402
from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer  # noqa: E402


def run(graph, autocast, rows, batches):
    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=16).cuda()
    w0 = {k: v.clone() for k, v in net.state_dict().items()}
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    tr = _Trainer(net, opt, memory_size=1000, batch_size=64, min_memory=0, q_average=True, device="cuda",
                  overlap=False, autocast=autocast, train_mode=False, graph=graph)
    tr.memory.add_moves(rows)
    for i, b in enumerate(batches):
        if i == 6:
            opt.param_groups[0]["lr"] = 0.002
        tr._step_graphed(*b) if graph else tr._train_step(*b)
    torch.cuda.synchronize()
    return {k: (v - w0[k]).double() for k, v in net.state_dict().items() if v.is_floating_point()}, tr


def rel(a, b):
    r = {k: ((a[k] - b[k]).norm() / (a[k].norm() + 1e-12)).item() for k in a}
    v = sorted(r.values())
    return {"max": v[-1], "median": v[len(v) // 2], "argmax": max(r, key=r.get)}


if "--deterministic" in sys.argv:
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
g = torch.Generator().manual_seed(7)
rows = dict(state=torch.randint(-1, 2, (512, 42), dtype=torch.int8, generator=g),
            tree_probs=torch.softmax(torch.randn(512, 7, generator=g), 1),
            q=torch.rand(512, dtype=torch.float64, generator=g) - 0.5,
            z=torch.randint(-1, 2, (512,), generator=g).float())
out = {}
for autocast in (False, True):
    torch.manual_seed(0)
    _, t = run(False, autocast, rows, [])
    torch.manual_seed(11)
    batches = [t.memory.sample_batch(64) for _ in range(10)]
    e1, _ = run(False, autocast, rows, batches)
    e2, _ = run(False, autocast, rows, batches)
    g1, _ = run(True, autocast, rows, batches)
    g2, _ = run(True, autocast, rows, batches)
    out["autocast" if autocast else "fp32"] = {"eager_vs_eager": rel(e1, e2), "graph_vs_graph": rel(g1, g2),
                                               "eager_vs_graph": rel(e1, g1)}
out["deterministic"] = "--deterministic" in sys.argv
print(json.dumps(out, indent=1))
