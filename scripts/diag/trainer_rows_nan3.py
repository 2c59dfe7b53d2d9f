"""The failing configuration alone in a fresh process (rows, trainer stream, graph, fp16 autocast, train
mode): the loss of each of 8 steps and the first step with a non-finite weight or buffer.
    python scripts/diag/trainer_rows_nan3.py [graph 0|1] [overlap 0|1]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from self_play_reinforcement_learning_amd.modules import ResidualTower
from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

graph = bool(int(sys.argv[1])) if len(sys.argv) > 1 else True
overlap = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
torch.manual_seed(0)
net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=16).cuda()
tr = _Trainer(net, torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9), memory_size=1000, batch_size=64,
              min_memory=0, q_average=True, device="cuda", overlap=overlap, autocast=True, graph=graph)
g = torch.Generator().manual_seed(1)
tr.memory.add_moves(dict(state=torch.randint(-1, 2, (256, 42), dtype=torch.int8, generator=g),
                         tree_probs=torch.full((256, 7), 1 / 7), q=torch.zeros(256, dtype=torch.float64),
                         z=torch.randint(-1, 2, (256,), generator=g).float()))
losses, bad = [], None
for i in range(8):
    loss = tr.step()
    tr.sync()
    torch.cuda.synchronize()
    losses.append(round(float(loss), 4))
    nf = [n for n, p in net.named_parameters() if not torch.isfinite(p).all()]
    nb = [n for n, b in net.named_buffers() if b.is_floating_point() and not torch.isfinite(b).all()]
    if (nf or nb) and bad is None:
        bad = (i, nf[:4], nb[:4])
print("graph", graph, "overlap", overlap, "hipblaslt", os.environ.get("TORCH_BLAS_PREFER_HIPBLASLT", "default"),
      losses, "first non-finite", bad, flush=True)
