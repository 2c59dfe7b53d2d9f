"""Multi-rank rehearsal on one GPU (torchrun, gloo): the scheduler's train_model + compare_models
with games sharded over ranks (per-ply Move gather / stats all_reduce / weight broadcast).
Run: SPMCTS_DIST_BACKEND=gloo torchrun --nproc-per-node 2 --master-addr 127.0.0.1 scripts/rehearse_multirank.py
"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from self_play_reinforcement_learning_amd import (Connect4Env, MCTreeSearch, ModelContainer, OneStepLookahead,
                                                  ResidualTower, SelfPlayScheduler)
from self_play_reinforcement_learning_amd import distributed as D

rank, world, local = D.init_from_env()
torch.manual_seed(0)
net = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=32)
container = ModelContainer(policy_gen=MCTreeSearch, policy_kwargs=dict(iterations=8, min_memory=64, batch_size=32,
                                                                        env=Connect4Env))
ev = ModelContainer(policy_gen=OneStepLookahead, policy_kwargs=dict(env=Connect4Env))
with tempfile.TemporaryDirectory() as d:
    sp = SelfPlayScheduler(policy_container=container, env=Connect4Env, network=net, evaluation_policy_container=ev,
                           initial_games=24, epoch_length=20, evaluation_games=10, save_dir=d, n_games=8,
                           lanes=int(os.environ.get("LANES", 2)))
    sp.train_model(2)
    total, breakdown = sp.compare_models()
mem = len(sp.trainer.memory) if sp.trainer is not None else -1
out = dict(rank=rank, world=world, games_done=sp.engine.games_done, memory=mem, compare_total=int(total),
           compare_games=sum(v for s in breakdown.values() for v in s.values()))
print(json.dumps(out), flush=True)
D.barrier()
if D.is_distributed():
    torch.distributed.destroy_process_group()
