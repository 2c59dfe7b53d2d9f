"""test_trainer_graph_train_mode_replays_run's setting (2 blocks, filter_factor 16, batch 64, SGD lr 0.01
momentum 0.9, fp16 autocast, train mode) over (rows, overlap, graph): the loss of each of 8 steps and
the first step with a non-finite weight."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from self_play_reinforcement_learning_amd.modules import ResidualTower
from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

for rows in (False, True):
    for overlap in (False, True):
        for graph in (False, True):
            torch.manual_seed(0)
            net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=16).cuda()
            tr = _Trainer(net, torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9), memory_size=1000,
                          batch_size=64, min_memory=0, q_average=True, device="cuda", overlap=overlap, autocast=True,
                          graph=graph, gemm_convs=rows)
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
            print("rows", rows, "overlap", overlap, "graph", graph, losses, "first non-finite", bad, flush=True)
