"""train_model throughput: self-play positions/s with the trainer on (SelfPlayScheduler's own loop:
`updates_per_ply` AZ-loss SGD steps queued after every ply, updateworker.py:141-149), plus SGD steps/s.

Workload: BASELINE configs[1] (Connect4, 200 sims, 4,096 games, ResNet-128x20, K = 4, two lanes) with
the reference's trainer settings (batch 64, SGD lr 0.001 momentum 0.9 wd 1e-4, min_memory 20,000,
memory 200,000).  `trainer_only`: ms per SGD step of the trainer alone (the update captured as one HIP
graph, the default, or eager; fp16 autocast as the UpdateWorker, or fp32).  `runs`: the replay ring is
first filled past min_memory (untimed), then --plies plies are timed with the trainer stepping (graphed
steps on their own stream, the default; eager steps; steps on the arena's stream), and once with
updates_per_ply = 0 for the self-play-only rate.

    python scripts/bench_train.py [--plies 24] [--updates 4]   -> one JSON line
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(args, updates, overlap, autocast=True, graph=True, hip_convs=True):
    import torch

    from self_play_reinforcement_learning_amd import Connect4Env, MCTreeSearch, ModelContainer, SelfPlayScheduler
    from self_play_reinforcement_learning_amd.modules import ResidualTower

    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32).cuda()
    kw = dict(iterations=args.sims, env=Connect4Env, batch_size=64, memory_size=200000, min_memory=args.min_memory)
    sp = SelfPlayScheduler(ModelContainer(MCTreeSearch, policy_kwargs=kw), Connect4Env, network=net, save_dir=None,
                           n_games=args.games, updates_per_ply=updates, overlap_training=overlap, evaluation_games=0,
                           train_autocast=autocast, train_graph=graph, train_hip_convs=hip_convs,
                           lr=0.001)
    sp.setup_player_workers()
    sp.setup_update_worker()
    eng, tr = sp.engine, sp.trainer
    on_moves, on_ply = sp._callbacks(update=True)
    eng.start()
    fill_plies = 0
    while len(tr.memory) < args.min_memory + 1000:  # untimed: the ring past min_memory (trainer starts)
        eng.ply(on_moves=on_moves)
        fill_plies += 1
    for _ in range(2):  # warm the trainer's kernels
        eng.ply(on_moves=on_moves)
        on_ply(eng)
    tr.sync()
    torch.cuda.synchronize()
    m0, s0 = eng.counters()["moves"], tr.steps
    t0 = time.perf_counter()
    for _ in range(args.plies):
        eng.ply(on_moves=on_moves)
        on_ply(eng)
    tr.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    moves, steps = eng.counters()["moves"] - m0, tr.steps - s0
    loss = float(tr.last_loss) if tr.last_loss is not None else None
    return dict(updates_per_ply=updates, trainer_stream=tr.stream is not None, train_autocast=autocast, train_graph=graph,
                train_hip_convs=tr.hip_convs,
                graph_captures=tr.graph_captures, plies=args.plies, seconds=dt,
                positions_per_s=moves / dt, sgd_steps=steps, sgd_steps_per_s=steps / dt, fill_plies=fill_plies,
                replay_rows=len(tr.memory), last_loss=loss)


def trainer_only(args, graph, autocast=True, steps=40, channels_last=False, benchmark=False, hip_convs=True):
    """ms per SGD step of the trainer alone (batch 64, ResNet-128x20, train mode), graphed or eager;
    `channels_last`: the network's tensors in NHWC order; `benchmark`: MIOpen's exhaustive kernel search
    (torch.backends.cudnn.benchmark); `hip_convs`: the residual blocks' 3x3 convolutions on the HIP
    matrix-core kernels (trainconv.py; under autocast only) instead of MIOpen."""
    import torch

    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

    torch.backends.cudnn.benchmark = bool(benchmark)
    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32).cuda()
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    tr = _Trainer(net, torch.optim.SGD(net.parameters(), lr=0.001, momentum=0.9, weight_decay=1e-4), memory_size=200000,
                  batch_size=64, min_memory=0, q_average=True, device="cuda", overlap=True, autocast=autocast,
                  graph=graph, hip_convs=hip_convs)
    g = torch.Generator().manual_seed(0)
    n = 20000
    tr.memory.add_moves(dict(state=torch.randint(-1, 2, (n, 42), dtype=torch.int8, generator=g),
                             tree_probs=torch.softmax(torch.randn(n, 7, generator=g), 1),
                             q=torch.rand(n, dtype=torch.float64, generator=g), z=torch.randint(-1, 2, (n,), generator=g).float()))
    for _ in range(6):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    tr.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    torch.backends.cudnn.benchmark = False
    return dict(train_graph=graph, train_autocast=autocast, train_hip_convs=tr.hip_convs, channels_last=channels_last,
                benchmark=benchmark, steps=steps,
                ms_per_sgd_step=dt / steps * 1e3, graph_captures=tr.graph_captures, last_loss=float(tr.last_loss))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plies", type=int, default=24)
    ap.add_argument("--updates", type=int, default=4)
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--min-memory", type=int, default=20000)
    ap.add_argument("--trainer-variants", action="store_true",
                    help="trainer-only timings of graphed steps with NHWC tensors and MIOpen's exhaustive search, "
                         "no self-play runs")
    ap.add_argument("--trainer-only-graph", action="store_true",
                    help="only the graphed fp16-autocast trainer-only timing (for a kernel trace)")
    ap.add_argument("--miopen-convs", action="store_true", help="with --trainer-only-graph: MIOpen's block convs")
    ap.add_argument("--conv-ab", action="store_true",
                    help="graphed autocast trainer-only timings, HIP block convs vs MIOpen, alternated 3 times")
    args = ap.parse_args()
    if args.trainer_only_graph:
        print(json.dumps(dict(trainer_only=[trainer_only(args, True, steps=100, hip_convs=not args.miopen_convs)])),
              flush=True)
        return
    if args.conv_ab:
        rows = [trainer_only(args, True, steps=100, hip_convs=h) for _ in range(3) for h in (True, False)]
        print(json.dumps(dict(trainer_only=rows)), flush=True)
        return
    if args.trainer_variants:
        rows = [trainer_only(args, True, autocast=a, channels_last=c, benchmark=b)
                for a in (True, False) for c in (False, True) for b in (False, True)]
        print(json.dumps(dict(trainer_only=rows)), flush=True)
        return
    out = dict(workload=f"connect4 self-play + training, {args.sims} sims, {args.games} games, ResNet-128x20 (fp16 "
                        f"fused trunk for leaves, the bench default; SGD batch 64 under fp16 autocast as "
                        f"updateworker.py:148), K = 4, two lanes",
               trainer_only=[trainer_only(args, True), trainer_only(args, True, hip_convs=False),
                             trainer_only(args, False)],
               runs=[run(args, args.updates, False), run(args, args.updates, False, hip_convs=False),
                     run(args, args.updates, True), run(args, 0, False)])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
