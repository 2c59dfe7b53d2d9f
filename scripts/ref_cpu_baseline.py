"""CPU-baseline calibration (build container only; needs /root/reference): the reference's OWN self-play
pipeline timed next to bench.py's cpu_baseline leg (the oracle "port") on the same host cores.

    python scripts/ref_cpu_baseline.py [seconds] [cores]

Reference side: SelfPlayScheduler.setup_player_workers(num_workers=cores,
threads_per_worker=8) — cores - 2 SelfPlayWorker processes x 8 game threads x MCTreeSearch(thread_count=4)
behind the InferenceWorker process (self_play_parallel.py:95-171, inference_worker.py:89-119) — with
ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32) (torch.manual_seed(0)), Connect4, 200 sims/move,
self-play tasks {"play": {"swap_sides": i % 2, "update": True}} as train_model issues them
(self_play_parallel.py:236-238).  Positions/s = moves played (MCTreeSearch._play calls, counted in the
worker processes through a shared counter) per second of the window, after a warm-up.

Port side: bench.cpu_baseline(..., cores, 200, 32, 20, threads=4) — bench.py's own leg, once with games
from the empty board (the same positions the reference's window sees; this gives the ratio) and once in
bench mode (random 0-16-move openings).

Writes profiles/r02/cpu_calibration.json; bench.py reads it to put a `calibration` field (the
port -> reference ratio on the same cores) next to its cpu_baseline on the GPU box.
"""
import json
import os
import sys
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden", "refshims"))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, REPO)

_tb = types.ModuleType("torch.utils.tensorboard")  # not installed: a no-op stand-in (logging only)


class _Writer:
    def __init__(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass


_tb.SummaryWriter = _Writer
sys.modules["torch.utils.tensorboard"] = _tb

from games.algos.mcts import MCTreeSearch  # noqa: E402


class CountingMCTS(MCTreeSearch):
    """The reference's MCTreeSearch; every _play (one position searched and played) bumps a
    counter shared with the harness."""

    def __init__(self, *a, move_counter=None, **k):
        self._move_counter = move_counter
        super().__init__(*a, **k)

    def _play(self, temp=0.05):
        a = super()._play(temp)
        if self._move_counter is not None:
            with self._move_counter.get_lock():
                self._move_counter.value += 1
        return a


def reference_rate(seconds, cores, warmup=30.0):
    import torch
    from torch import multiprocessing

    from games.algos.self_play_parallel import SelfPlayScheduler
    from games.connect4.connect4env import Connect4Env
    from games.general.base_model import ModelContainer
    from games.general.modules import ResidualTower

    counter = multiprocessing.Value("l", 0)
    torch.manual_seed(0)
    net = ResidualTower(width=7, height=6, action_size=7, num_blocks=20, filter_factor=32)
    container = ModelContainer(CountingMCTS, policy_kwargs=dict(env=Connect4Env, network=net, iterations=200,
                                                                thread_count=4, move_counter=counter))
    os.makedirs("/tmp/ref_cpu_saves", exist_ok=True)
    from games.general.hardcoded_players import OneStepLookahead

    # an opponent container as main.py's train() passes (main.py:64-70, :81-100); its policy_kwargs hold
    # no network, so no evaluation proxies are built (setup_player_workers dereferences it)
    opponent = ModelContainer(OneStepLookahead, policy_kwargs=dict(env=Connect4Env))
    sched = SelfPlayScheduler(container, Connect4Env, evaluation_policy_container=opponent,
                              save_dir="/tmp/ref_cpu_saves", epoch_length=10_000)
    workers, inference, _ = sched.setup_player_workers(num_workers=cores, threads_per_worker=8)
    for w in workers:
        w.start()
    for i in range(400):
        sched.task_queue.put({"play": {"swap_sides": not i % 2 == 0, "update": True}})
    time.sleep(warmup)
    c0, t0 = counter.value, time.time()
    time.sleep(seconds)
    c1, t1 = counter.value, time.time()
    for p in workers + [inference]:
        p.terminate()
    return dict(value=(c1 - c0) / (t1 - t0), moves=c1 - c0, seconds=t1 - t0, warmup_s=warmup,
                play_workers=len(workers), threads_per_worker=8, thread_count=4, cores=cores)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    cores = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 8)
    from torch import multiprocessing

    multiprocessing.set_start_method("spawn", force=True)  # the reference's own start method (main.py:109)
    os.chdir("/tmp")
    ref = reference_rate(seconds, cores)
    print("reference", json.dumps(ref), flush=True)
    sys.path.insert(0, REPO)
    import bench

    port = bench.cpu_baseline(seconds / 3, cores, 200, 32, 20, threads=4, openings=False)
    print("port (empty-board games, like the reference's window)", json.dumps(port), flush=True)
    port_mid = bench.cpu_baseline(seconds / 3, cores, 200, 32, 20, threads=4, openings=True)
    print("port (bench mode: random openings)", json.dumps(port_mid), flush=True)
    out = dict(reference=ref, port=port, port_bench_mode=port_mid,
               ratio_reference_over_port=ref["value"] / port["value"], cores=cores,
               host=os.uname().nodename, note="same host, same cores, run back to back, both from the empty board: "
               "the reference's full multiprocess pipeline (InferenceWorker + play workers) vs bench.py's "
               "cpu_baseline leg; the ratio maps the bench's port figure to the reference's pipeline")
    os.makedirs(os.path.join(REPO, "profiles", "r02"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r02", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
