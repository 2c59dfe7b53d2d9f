"""`SelfPlayScheduler` with the reference API, driving the device arena.

Drop-in for games/algos/self_play_parallel.py:44-379.  The constructor takes
the same arguments (plus the stale `self_play=` its own callers pass,
run_self_play_connect4.py:61, elo.py:81), and `train_model`,
`compare_models`, `evaluate_policy`, `run_evaluation_games`,
`parse_results`, `setup_player_workers`, `setup_update_worker` keep their
signatures.  What changes is underneath:

  * instead of (cpu_count - 2) SelfPlayWorker processes x threads_per_worker
    games x thread_count search threads + an InferenceWorker over
    multiprocessing queues, ONE SelfPlayEngine per GPU runs `n_games`
    concurrent games in lock step (all leaves of all games = one network
    batch);
  * the memory queue, result queue and task queue are in-process objects with
    the same put/get/empty surface (results carry the reference's
    {"reward", "swap_sides"} dicts, moves are `Move` namedtuples);
  * the UpdateWorker's training (updateworker.py:141-149: AlphaZero loss, SGD
    lr/momentum 0.9/wd 1e-4, 100 steps per update call, checkpoint
    {"model": state_dict} per epoch, LR on plateau) runs in-process between
    plies on the same GPU; self-play uses the epoch-start weights, refreshed at
    each epoch boundary exactly like the reference's epoch_value reload.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE > 1) every rank plays
its own shard of games; Move records and episode statistics are gathered to
rank 0 (distributed.py).  Without torchrun, `train_model` / `compare_models`
start the rank processes themselves when asked (`gpus=N` or `gpus="all"`; the
default runs in this process, on the constructor's device), as
the reference's scheduler starts its own worker processes
(self_play_parallel.py:95-171, num_workers = cpu_count()): the children rebuild
this scheduler from its constructor arguments (networks copied to the host),
rank 0 checkpoints, and the parent's network is updated from the last
checkpoint afterwards, as the reference's shared-memory network is updated by
its UpdateWorker process.
"""
import copy
import datetime
import logging
import os
import time
from collections import deque

import numpy as np
import torch

from . import distributed as D
from .arena import GAMES, game_of_env
from .engine import LanedEngine, SelfPlayEngine
from .mcts import MCTreeSearch, Move, az_loss


class LocalQueue:
    """In-process stand-in for the multiprocessing queues (put / get / empty / qsize)."""

    def __init__(self):
        self._q = deque()

    def put(self, item):
        self._q.append(item)

    def get(self, block=True, timeout=None):
        return self._q.popleft()

    def empty(self):
        return not self._q

    def qsize(self):
        return len(self._q)

    def join(self):
        pass

    def task_done(self):
        pass


def moves_to_records(moves, W, H):
    """Arena export rows -> Move namedtuples (mcts.py:17; dtypes as mcts.py:282-288, :230)."""
    st = moves["state"].cpu().numpy().astype(np.int64)
    tp = moves["tree_probs"].cpu()
    q = moves["q"].cpu().numpy()
    qf = moves["q_f64"].cpu().numpy()
    z = moves["z"].cpu()
    out = []
    for i in range(len(z)):
        qt = torch.tensor(float(q[i]), dtype=torch.float64 if qf[i] else torch.float32)
        out.append(Move(torch.as_tensor(st[i].reshape(W, H)), z[i].clone(), tp[i].clone(), qt))
    return out


class SelfPlayScheduler:
    def __init__(self, policy_container, env, evaluation_policy_container=None, network=None, swap_sides=True,
                 save_dir="saves", epoch_length=500, initial_games=64, lr=0.001, stagger=False, evaluation_games=100,
                 evaluation_network=None, stagger_mem_step=5000, deduplicate=False, update_delay=0.01,
                 self_play=None, n_games=None, device=None, seed=0, updates_per_ply=4, lanes=None, exchange_every=8,
                 gpus=None, start_time=None, overlap_training=False, train_autocast=True, train_graph=True,
                 train_hip_convs=True):
        # constructor arguments, for rank processes started by this scheduler (_run_ranks)
        self._init_kwargs = {k: v for k, v in locals().items() if k not in ("self", "__class__")}
        self.policy_container = policy_container
        self.evaluation_policy_container = evaluation_policy_container
        self.env_gen = env
        self.game = game_of_env(env)
        _, self.W, self.H, self.A = GAMES[self.game]
        self.swap_sides = swap_sides
        self.save_dir = save_dir
        self.epoch_length = epoch_length
        self.initial_games = initial_games
        self.lr = lr
        self.stagger = stagger
        self.stagger_mem_step = stagger_mem_step
        self.deduplicate = deduplicate
        self.update_delay = update_delay
        self.evaluation_games = evaluation_games
        self.evaluation_network = evaluation_network
        self.network = self._get_network(network, policy_container)
        self.seed = seed
        self.updates_per_ply = updates_per_ply
        # True: the trainer's SGD steps on a HIP stream of their own, beside the arena's plies (_Trainer).
        # Off by default: with the graphed step the arena keeps the GPU busy either way and the steps
        # ordered on the plies' stream measured faster (18.1k vs 17.7k positions/s at 4 steps per ply,
        # profiles/r04/trainer/train_throughput.json)
        self.overlap_training = overlap_training
        # the UpdateWorker's update_from_memory runs under torch.cuda.amp.autocast() (fp16 on CUDA, no
        # GradScaler; updateworker.py:148); False trains in fp32
        self.train_autocast = train_autocast
        # the trainer's update captured as one HIP graph and replayed per step (_Trainer graph=True)
        self.train_graph = train_graph
        # the residual blocks' 3x3 convolutions of the autocast update on the HIP matrix-core kernels
        # (trainconv.py) instead of MIOpen (_Trainer hip_convs=True)
        self.train_hip_convs = train_hip_convs
        self.exchange_every = exchange_every  # plies per episode-batch exchange round (distributed.MoveExchange)
        # >1: LanedEngine (arenas on separate HIP streams, each a complete arena); None = 2 lanes for
        # arenas of >= 1,024 games, where the overlap pays (bench.py), else one arena
        self.lanes = None if lanes is None else max(1, int(lanes))
        if D.in_launched_job() and int(D.env_rank()[1]) > 1:
            D.init_from_env()  # one rank of a torchrun / self-launched job
        rank, world, local = D.env_rank()
        self.rank, self.world = rank, world
        self.gpus = gpus
        self.device = torch.device(device) if device is not None else D.local_device()
        self.n_games = n_games
        self.start_time = start_time or datetime.datetime.now().isoformat()
        self.task_queue = LocalQueue()
        self.memory_queue = LocalQueue()
        self.result_queue = LocalQueue()
        self.engine = None
        self.trainer = None
        self.epoch_value = 0
        self._search_threads = self._opponent_threads = 1
        if policy_container is not None:
            self._resolve_threads(True)  # the default of every entry point (inference_proxy=True)
        if save_dir and rank == 0:
            os.makedirs(os.path.join(save_dir, self.start_time), exist_ok=True)

    # ------------------------------------------------------------------ reference helpers
    def _get_network(self, network, container):
        """self_play_parallel.py:173-184"""
        if network is not None:
            return network
        if container is None:
            return None
        if container.policy_kwargs.get("network") is not None:
            return container.policy_kwargs.pop("network")
        if container.policy_kwargs.get("evaluator") is not None:  # deprecated key
            return container.policy_kwargs.pop("evaluator")
        return None

    def _policy_kwargs(self):
        kw = dict(self.policy_container.policy_kwargs)
        return kw

    def _resolve_threads(self, inference_proxy=True):
        """Simulations in flight per tree, resolved in one place for self-play and evaluation
        games: the reference's workers search with thread_count threads + virtual loss exactly when
        they talk to an InferenceProxy (mcts.py:154, self_play_parallel.py:95-171), which every
        scheduler entry point does by default.  The evaluation opponent is built from its own
        container's kwargs (selfplayworker.py:71-81), so it searches with its own thread_count."""
        def threads(kw):
            return max(1, int(kw.get("thread_count", 4) or 1)) if inference_proxy else 1

        k = threads(self._policy_kwargs())
        okw = getattr(self.evaluation_policy_container, "policy_kwargs", None) or {}
        self._search_threads = k
        self._opponent_threads = threads(okw)
        return k

    def setup_player_workers(self, num_workers=None, inference_proxy=True, threads_per_worker=8, resume_model=False):
        """Build the device self-play engine (replaces the worker processes, :95-171)."""
        kw = self._policy_kwargs()
        n_games = self.n_games or max(64, min(4096, (num_workers or 1) * threads_per_worker * 64))
        if resume_model:
            self._load_latest(prev_run=True)
        threads = self._resolve_threads(inference_proxy)
        ekw = dict(iterations=kw.get("iterations", 100), alpha=kw.get("alpha", 1),
                   strong_play=kw.get("strong_play", False), seed=self.seed + 7919 * self.rank, device=self.device,
                   search_threads=max(1, threads))
        lanes = self.lanes if self.lanes is not None else (2 if n_games >= 1024 else 1)
        if lanes > 1 and n_games >= 2 * lanes:
            self.engine = LanedEngine(self.game, self.network, n_games=n_games, lanes=lanes, **ekw)
        else:
            self.engine = SelfPlayEngine(self.game, self.network, n_games=n_games, **ekw)
        return self.engine, None, self.epoch_value

    def setup_update_worker(self, resume_memory=False, resume_model=False):
        """The trainer (updateworker.py:16-149) as an in-process MCTreeSearch-style policy."""
        kw = self._policy_kwargs()
        self.network.to(self.device)
        optim = torch.optim.SGD(self.network.parameters(), weight_decay=0.0001, momentum=0.9, lr=self.lr)
        self.trainer = _Trainer(self.network, optim, memory_size=kw.get("memory_size", 200000),
                                batch_size=kw.get("batch_size", 64), min_memory=kw.get("min_memory", 20000),
                                q_average=kw.get("q_average", True), device=self.device, W=self.W, H=self.H,
                                A=self.A, overlap=self._overlap_ok(), autocast=self.train_autocast,
                                graph=self.train_graph, hip_convs=self.train_hip_convs)
        if self.save_dir and self.rank == 0:  # rank 0 owns the replay ring (MoveExchange gathers to it)
            self.trainer.run_dir = os.path.join(self.save_dir, self.start_time)
        if resume_memory and self.rank == 0:  # updateworker.py:67-69 (before the model, as there)
            self._load_memory(prev_run=True)
        if resume_model:
            self._load_latest(prev_run=True)
        return self.trainer, None, None

    def _load_memory(self, prev_run=False):
        """BaseWorker.load_memory (base_worker.py:36-41, recent_save_file :44-62): the newest `memory*`
        snapshot of the newest non-empty run folder (other than this run's with prev_run) replaces the
        trainer's replay ring.  The reference's max() over no folder raises, which its UpdateWorker logs
        (updateworker.py:76-78); here that is a warning and the ring stays empty."""
        from glob import glob

        if not self.save_dir:
            logging.warning("resume_memory: no save_dir; starting from an empty replay")
            return None
        runs = sorted(d for d in glob(os.path.join(self.save_dir, "*")) if os.path.isdir(d)
                      and (not prev_run or os.path.basename(d) != self.start_time) and os.listdir(d))
        saves = sorted(glob(os.path.join(runs[-1], "memory*"))) if runs else []
        if not saves:
            logging.warning(f"resume_memory: no memory snapshot under {self.save_dir}; starting from an empty replay")
            return None
        self.trainer.load_memory(saves[-1])
        return saves[-1]

    def _overlap_ok(self):
        """SGD steps on the trainer's own stream beside the plies only when the self-play engine's
        evaluators hold a snapshot of the weights (the fused HIP trunk's packed blobs, a bf16 / fp16
        folded tower): an evaluator that reads the live module (ModuleEvaluator, an fp32 folded tower)
        would race with optimizer.step, so its steps stay on the plies' stream, in order."""
        eng = self.engine
        return bool(self.overlap_training and eng is not None and getattr(eng, "weights_snapshot", False))

    def _load_latest(self, prev_run=False):
        from glob import glob

        if not self.save_dir:
            return None
        runs = sorted(d for d in glob(os.path.join(self.save_dir, "*")) if os.path.isdir(d)
                      and (not prev_run or os.path.basename(d) != self.start_time) and os.listdir(d))
        if not runs:
            return None
        return self._load_checkpoint(runs[-1])

    def _load_checkpoint(self, run_dir):
        """The newest `model-<iso>:<games>` of one run folder (base_worker.py:44-62) into the network."""
        from glob import glob

        saves = sorted(glob(os.path.join(run_dir, "model*")))
        if not saves:
            return None
        ck = torch.load(saves[-1], weights_only=True, map_location="cpu")
        self.network.load_state_dict(ck["model"])
        return saves[-1]

    # ------------------------------------------------------------------ self-play
    def _play_games(self, n_games, update=True):
        """Play `n_games` self-play games over all ranks (task ids i -> swap_sides = i odd,
        self_play_parallel.py:236-238); Moves -> memory_queue (rank 0), results -> result_queue."""
        eng = self.engine
        per_rank = n_games // self.world + (1 if self.rank < n_games % self.world else 0)
        on_moves, on_ply = self._callbacks(update)
        eng.play_games(per_rank, on_moves=on_moves, on_ply=on_ply, every=self.exchange_every)
        eng.check()

    def _callbacks(self, update=True):
        """(on_moves, on_ply) of a self-play run: gathered Move rows into the replay ring (rank 0) and
        the results queue; `updates_per_ply` trainer steps queued after every ply."""

        def on_moves(g):
            # rank 0 (the replay owner): a batch of Move rows gathered from every rank (MoveExchange)
            if update and self.trainer is not None:
                self.trainer.sync()  # queued SGD steps sample the ring: they finish before rows are overwritten
                self.trainer.memory.add_moves(g)  # device replay ring: no per-record host objects
                self.trainer.rows_added()  # a snapshot every 50,000 positions (UpdateWorker.pull)
            elif update:
                for rec in moves_to_records(g, self.W, self.H):
                    self.memory_queue.put(rec)
            first = {}
            for gid, z in zip(g["game"].cpu().tolist(), g["z"].cpu().tolist()):
                first.setdefault(gid, z)  # the policy's Moves come first: z = r (policy's view)
            for gid, z in first.items():
                self.result_queue.put({"reward": int(z), "swap_sides": bool(gid % 2)})

        def on_ply(_):
            if update and self.trainer is not None:
                self.trainer.pull(self.memory_queue)
                for _ in range(self.updates_per_ply):
                    self.trainer.step()

        return on_moves, on_ply

    # ------------------------------------------------------------------ one process per GPU
    def _ranks(self, gpus):
        """How many rank processes this call starts: 1 (run here) inside a launched job; else `gpus`
        (the call's, then the constructor's; None = 1, in this process on the constructor's device;
        "all" = every visible GPU).  After a multi-rank run this scheduler holds no trainer or engine
        state: only its network, loaded from the last checkpoint (train_model)."""
        if D.in_launched_job() or D.is_distributed():
            return 1
        n = gpus if gpus is not None else self.gpus
        if n is None:
            return 1
        if n == "all":
            n = torch.cuda.device_count()  # counting devices does not initialise the GPU
        return max(1, int(n))

    def _spawn_kwargs(self):
        """Constructor arguments for the rank processes: modules copied to the host (CPU tensors travel
        to spawned processes by shared memory), the same start_time (one checkpoint folder)."""
        def host(obj):
            if isinstance(obj, torch.nn.Module):
                return copy.deepcopy(obj).cpu()
            if isinstance(obj, dict):
                return {k: host(v) for k, v in obj.items()}
            if isinstance(obj, (list, tuple)):
                return type(obj)(host(v) for v in obj)
            if hasattr(obj, "policy_kwargs"):  # ModelContainer
                c = copy.copy(obj)
                c.policy_kwargs = host(obj.policy_kwargs)
                return c
            return obj

        kw = {k: host(v) for k, v in self._init_kwargs.items()}
        kw.update(network=host(self.network), start_time=self.start_time, device=None, gpus=1)
        return kw

    def _run_ranks(self, n, method, kwargs):
        D.check_devices(n)
        import multiprocessing as mp

        q = mp.get_context("spawn").Queue()
        D.spawn_ranks(_scheduler_rank, n, self._spawn_kwargs(), method, kwargs, q)
        return q.get(timeout=60)

    def train_model(self, num_epochs=10, resume_model=False, resume_memory=False, num_workers=None,
                    threads_per_worker=8, inference_proxy=True, gpus=None):
        """self_play_parallel.py:213-291.  gpus > 1 (or "all") outside a launched job: one rank process
        per GPU (_run_ranks); this scheduler's network then holds the final checkpoint's weights."""
        n = self._ranks(gpus)
        if n > 1:
            self._run_ranks(n, "train_model", dict(num_epochs=num_epochs, resume_model=resume_model,
                                                    resume_memory=resume_memory, num_workers=num_workers,
                                                    threads_per_worker=threads_per_worker,
                                                    inference_proxy=inference_proxy))
            self._load_checkpoint(os.path.join(self.save_dir, self.start_time))
            return None
        self.setup_player_workers(num_workers=num_workers, threads_per_worker=threads_per_worker,
                                  resume_model=resume_model, inference_proxy=inference_proxy)
        self.setup_update_worker(resume_memory=resume_memory, resume_model=resume_model)
        logging.info(f"generating {self.initial_games} initial games")
        self._play_games(self.initial_games, update=True)
        while not self.result_queue.empty():
            self.result_queue.get()
        if self.evaluation_games:
            self.evaluate_policy(-1)
        for epoch in range(num_epochs):
            self._play_games(self.epoch_length, update=True)
            saved = os.path.join(self.save_dir, self.start_time,
                                 "model-" + datetime.datetime.now().isoformat() + ":" + str(self.epoch_length * (epoch + 1)))
            self.trainer.sync()  # the weights after every queued SGD step
            if self.rank == 0:
                torch.save({"model": self.network.state_dict()}, saved)
            D.broadcast_state_dict(self.network)
            self.engine.refresh_network()  # epoch_value reload (selfplayworker.py:109-114)
            self.epoch_value += 1
            if self.stagger:  # UpdateWorker.stagger_memory (updateworker.py:107-109)
                m = self.trainer.memory
                m.change_size(min(m.max_size + self.stagger_mem_step, 1500000))
            if self.deduplicate:
                if epoch == 0:
                    logging.warning("deduplicate=True merges duplicate boards of the replay ring; the reference's "
                                    "own deduplicate() raises TypeError with its Move type (memory.py:93) and merges "
                                    "nothing, so training data differs from the reference's from here on")
                # updateworker.py:88-89 calls policy.deduplicate() here; with the reference's own Move
                # that raises TypeError (memory.py:93: the rebuilt tuple lacks q) and, caught, skips the
                # checkpoint.  The device ring merges duplicate boards (z, tree_probs and q averaged);
                # its (state, z, tree_probs) part is pinned by G7 (tests/test_memory_golden.py)
                self.trainer.memory.deduplicate()
            self.trainer.save_memory()  # updateworker.py:92, after stagger / dedup (:86-89)
            reward = self.evaluate_policy(epoch)
            self.trainer.lr_step(reward)

    # ------------------------------------------------------------------ evaluation games
    def _opponent(self):
        """The evaluation side of SelfPlayWorker.set_up_policies(evaluate=True) (selfplayworker.py:72-81):
        (opponent for SelfPlayEngine, its iterations)."""
        c = self.evaluation_policy_container
        if c is None:
            raise ValueError("evaluation games need an evaluation_policy_container")
        gen = getattr(c, "policy_gen", None)
        name = getattr(gen, "__name__", "").lower()
        if name in ("random", "onesteplookahead"):
            return ("random" if name == "random" else "lookahead"), {}
        kw = dict(getattr(c, "policy_kwargs", {}) or {})
        net = self.evaluation_network
        if net is None:
            net = kw.get("network", kw.get("evaluator"))
        if net is None:
            raise ValueError("the evaluation MCTreeSearch has no network (pass evaluation_network=)")
        # the opponent's own MCTreeSearch kwargs (mcts.py:119-136 defaults), per side in the arena
        return net, dict(opponent_iterations=kw.get("iterations", 100), opponent_alpha=kw.get("alpha", 1),
                         opponent_strong_play=kw.get("strong_play", False),
                         opponent_search_threads=self._opponent_threads)

    def _evaluation_engine(self, n_games):
        opponent, opp_kw = self._opponent()
        kw = self._policy_kwargs()
        per_rank = max(1, n_games // self.world + (1 if self.rank < n_games % self.world else 0))
        slots = min(per_rank, self.n_games or 4096)
        self.network.eval()
        return SelfPlayEngine(self.game, self.network, n_games=slots, iterations=kw.get("iterations", 100),
                              alpha=kw.get("alpha", 1), strong_play=kw.get("strong_play", False), evaluate=True,
                              seed=self.seed + 104729 + 7919 * self.rank, device=self.device, opponent=opponent,
                              record=False, search_threads=self._search_threads, **opp_kw), per_rank

    def _play_evaluation(self, n_games):
        """n_games evaluation games over all ranks (task i -> swap_sides = i odd, update=False);
        returns the reference's result dicts (self_play_parallel.py:294-300, :366-371)."""
        if n_games <= 0:
            return []
        eng, per_rank = self._evaluation_engine(n_games)
        c0 = eng.counters()["results"]
        eng.play_games(per_rank)
        eng.check()
        c1 = eng.counters()["results"]
        flat = [c1[s][k] - c0[s][k] for s in range(2) for k in range(3)]
        flat = [int(x) for x in D.all_reduce_stats(flat)]
        reward_list = []
        for s in range(2):
            for k, r in enumerate((1, 0, -1)):
                reward_list += [{"reward": r, "swap_sides": bool(s)}] * flat[3 * s + k]
        eng.arena.close()
        return reward_list

    def run_evaluation_games(self):
        """self_play_parallel.py:294-300: evaluation_games games of the policy against the
        evaluation policy (both in evaluate mode, no Move records); results -> result_queue."""
        if self.evaluation_policy_container is None or not self.evaluation_games:
            return
        for r in self._play_evaluation(self.evaluation_games):
            self.result_queue.put(r)

    def parse_results(self, reward_list):
        """self_play_parallel.py:302-327"""
        if not reward_list:
            return 0, {"first": dict(wins=0, draws=0, losses=0), "second": dict(wins=0, draws=0, losses=0)}
        win_percent = sum(1 if r["reward"] > 0 else 0 for r in reward_list) / len(reward_list) * 100
        wins = len([i for i in reward_list if i["reward"] == 1])
        draws = len([i for i in reward_list if i["reward"] == 0])
        losses = len([i for i in reward_list if i["reward"] == -1])
        print(f"win percent : {win_percent}%")
        print(f"wins: {wins}, draws: {draws}, losses: {losses}")
        breakdown = {}
        for j, start in enumerate(["first", "second"]):
            sel = [i for i in reward_list if i["swap_sides"] == bool(j)]
            breakdown[start] = dict(wins=len([i for i in sel if i["reward"] == 1]),
                                    draws=len([i for i in sel if i["reward"] == 0]),
                                    losses=len([i for i in sel if i["reward"] == -1]))
        total_rewards = int(np.sum([r["reward"] for r in reward_list]))
        return total_rewards, breakdown

    def evaluate_policy(self, epoch):
        """self_play_parallel.py:329-353: parse the self-play results, then play and parse evaluation games."""
        reward_list = []
        while not self.result_queue.empty():
            reward_list.append(self.result_queue.get())
        total = 0
        if epoch >= 0 and reward_list:
            total, _ = self.parse_results(reward_list)
        if self.evaluation_policy_container is None or not self.evaluation_games:
            return total
        self.run_evaluation_games()
        reward_list = []
        while not self.result_queue.empty():
            reward_list.append(self.result_queue.get())
        total, _ = self.parse_results(reward_list)
        return total

    def compare_models(self, num_workers=None, inference_proxy=True, threads_per_worker=8, resume_model=False,
                       gpus=None):
        """self_play_parallel.py:355-379: epoch_length evaluation games, policy network vs the
        evaluation policy (a second network on the same arena, or a hard-coded player).
        Returns (total_rewards, breakdown) exactly as the reference's parse_results; with gpus > 1
        the games are sharded over one rank process per GPU."""
        n = self._ranks(gpus)
        if n > 1:
            return self._run_ranks(n, "compare_models", dict(num_workers=num_workers, inference_proxy=inference_proxy,
                                                              threads_per_worker=threads_per_worker,
                                                              resume_model=resume_model))
        if resume_model:
            self._load_latest(prev_run=True)
        self._resolve_threads(inference_proxy)  # evaluation workers talk to the InferenceProxy too
        reward_list = self._play_evaluation(self.epoch_length)
        return self.parse_results(reward_list)


def _scheduler_rank(kwargs, method, call_kwargs, result_q):
    """One rank process of SelfPlayScheduler._run_ranks (the environment holds RANK / WORLD_SIZE)."""
    sp = SelfPlayScheduler(**kwargs)
    try:
        out = getattr(sp, method)(**call_kwargs)
        if sp.rank == 0:
            result_q.put(out)
    finally:
        if D.is_distributed():
            torch.distributed.destroy_process_group()


class _Trainer:
    """UpdateWorker core (updateworker.py:119-149) on the same device: AZ-loss SGD steps on batches
    sampled from the device replay ring (replay.DeviceReplay), LR on plateau.

    The reference's UpdateWorker trains in its own process while the workers play
    (updateworker.py:141-149).  Here `step()` enqueues the update on a HIP stream of its own and
    returns without a host synchronisation, so the SGD kernels run beside the arena's next ply
    (self-play evaluates leaves with its own packed copy of the epoch-start weights, refreshed at
    epoch boundaries).  `sync()` makes the current stream wait for the queued steps: before replay
    rows are overwritten and before the weights are read (checkpoint, weight refresh).

    `graph` (CUDA device, default on): after `GRAPH_WARMUP` eager steps the whole update -- forward,
    AZ loss, backward, SGD/momentum/weight-decay step, BatchNorm statistics, dropout -- is captured
    once as a HIP graph (torch.cuda.CUDAGraph) and replayed per step: one launch instead of ~600
    small kernels, whose launch costs dominated a batch-64 step of ResNet-128x20.  The sampled batch
    (uniform without replacement, on the device) is copied into the graph's static input buffers
    first.  The graph is re-captured when the learning rate changes (ReduceLROnPlateau), since the
    captured optimizer kernels hold the rate as a constant."""

    GRAPH_WARMUP = 3

    def __init__(self, network, optim, memory_size, batch_size, min_memory, q_average, device, W=7, H=6, A=7,
                 train_mode=True, overlap=True, autocast=False, graph=True, hip_convs=True):
        from .replay import DeviceReplay

        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.stream = torch.cuda.Stream(device=dev) if overlap and dev.type == "cuda" else None
        self.steps = 0
        self.last_loss = None  # device tensor of the latest queued step
        self.network = network
        self.optim = optim
        self.memory = DeviceReplay(memory_size, W, H, A, device=device)
        self.batch_size = batch_size
        self.min_memory = min_memory
        self.q_average = q_average
        self.device = device
        self.train_mode = train_mode  # the UpdateWorker trains in train mode (updateworker.py:63)
        # forward, loss and backward under fp16 autocast as the UpdateWorker (updateworker.py:147-149:
        # `with autocast(): self.policy.update_from_memory()`, no GradScaler); only on a CUDA device,
        # where the reference's autocast is active (it is a no-op on CPU)
        self.autocast = bool(autocast) and dev.type == "cuda"
        # under autocast the residual blocks' 3x3 convolutions (forward and backward) run on the HIP
        # matrix-core kernels (trainconv.py) instead of MIOpen's VALU Winograd kernels
        self.hip_convs = bool(hip_convs) and self.autocast
        self.scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optim, "max", patience=15, factor=0.5,
                                                                    min_lr=0.00001, cooldown=5)
        self.graph = bool(graph) and dev.type == "cuda"
        self._g = None          # the captured step (torch.cuda.CUDAGraph)
        self._g_key = None      # (lr of every param group, autocast, train_mode) it was captured with
        self._g_in = None       # its static inputs (s, z, pi, q)
        self._g_loss = None     # its static loss output
        self._eager_steps = 0   # eager steps since the last (re)capture request
        self.graph_captures = 0
        # replay snapshots (updateworker.py:51-53, :119-139): into run_dir (None = never), one kept
        self.run_dir = None
        self.memory_size = 0
        self.memory_size_step = 50000
        self.recent_save = None

    def pull(self, queue):
        while not queue.empty():
            self.memory.add(queue.get())
        self.rows_added()

    def rows_added(self):
        """UpdateWorker.pull's cadence (updateworker.py:119-125): a snapshot whenever the replay's
        length crosses a multiple of 50,000 (so none once the ring is full: its length stays at the
        capacity; the epoch-end snapshot still runs)."""
        n = len(self.memory)
        if n // self.memory_size_step - self.memory_size // self.memory_size_step > 0:
            self.memory_size = n
            self.save_memory()
        self.memory_size = n

    def save_memory(self):
        """UpdateWorker.save_memory (updateworker.py:127-139): `memory-<iso>:<length>` in the run folder,
        the previous snapshot removed.  The file holds tensors only (DeviceReplay.snapshot)."""
        if self.run_dir is None:
            return None
        os.makedirs(self.run_dir, exist_ok=True)
        name = os.path.join(self.run_dir, "memory-" + datetime.datetime.now().isoformat() + ":" + str(self.memory_size))
        self.sync()  # rows written on the plies' stream; queued SGD steps only read them
        tmp = os.path.join(self.run_dir, ".memory.partial")  # not matched by the loader's memory* glob
        self.memory.save(tmp)
        os.replace(tmp, name)
        if self.recent_save and self.recent_save != name and os.path.exists(self.recent_save):
            logging.info(f"removing {self.recent_save}")
            os.remove(self.recent_save)
        self.recent_save = name
        return name

    def load_memory(self, path):
        """BaseWorker.load_memory (base_worker.py:36-41): the snapshot replaces the ring."""
        self.memory.load(path)
        self.memory_size = len(self.memory)

    def step(self):
        """One update (mcts.py:254-270): uniform batch without replacement from the device ring.
        With a trainer stream: queued there (after the rows added so far), no host sync; returns
        the loss as a device tensor."""
        if len(self.memory) < max(self.batch_size, self.min_memory):
            return None
        self.steps += 1
        if self.stream is None:
            if self.graph:
                self.last_loss = self._step_graphed(*self.memory.sample_batch(self.batch_size))
                return float(self.last_loss)
            return self.train_batch(*self.memory.sample_batch(self.batch_size))
        self.stream.wait_stream(torch.cuda.current_stream(self.stream.device))
        with torch.cuda.stream(self.stream):
            batch = self.memory.sample_batch(self.batch_size)
            self.last_loss = self._step_graphed(*batch) if self.graph else self._train_step(*batch)
        return self.last_loss

    def sync(self):
        """The current stream waits for the queued training steps (GPU-side, no host sync)."""
        if self.stream is not None:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)

    def _train_step(self, s, z, pi, q):
        from .trainconv import hip_block_convs

        self.network.train(self.train_mode)
        with torch.autocast("cuda", dtype=torch.float16, enabled=self.autocast), \
                hip_block_convs(self.network, self.hip_convs):
            loss = az_loss(self.network, s, z, pi, q, self.q_average)
            self.optim.zero_grad()
            loss.backward()
            self.optim.step()
        self.network.eval()
        return loss.detach()

    def _graph_key(self):
        return (tuple(float(g["lr"]) for g in self.optim.param_groups), self.autocast, self.train_mode)

    def _step_graphed(self, s, z, pi, q):
        """One update through the captured graph (on the current stream).  The first GRAPH_WARMUP
        steps after a (re)capture request run eagerly -- they are real updates, and they create the
        optimizer's momentum buffers and let the convolution library settle its kernel choice -- then
        the update is captured and every later step is a copy of the batch + one graph replay."""
        key = self._graph_key()
        if self._g is not None and key != self._g_key:
            self._g = None  # learning rate changed: the captured SGD kernels hold the old one
            self._eager_steps = 0
        if self._g is None and self._eager_steps < self.GRAPH_WARMUP:
            self._eager_steps += 1
            return self._train_step(s, z, pi, q)
        if self._g is None:
            self._capture(s, z, pi, q)
            self._g_key = key
        for dst, src in zip(self._g_in, (s, z, pi, q)):
            dst.copy_(src)
        self._g.replay()
        self.network.eval()  # the captured step ran in train mode; module flags are host state
        return self._g_loss.detach().clone()  # the static output is overwritten by the next replay

    def _capture(self, s, z, pi, q):
        self._g_in = tuple(t.detach().clone() for t in (s, z, pi, q))
        g = torch.cuda.CUDAGraph()
        self.network.train(self.train_mode)
        self.optim.zero_grad(set_to_none=True)  # the gradients are allocated inside the graph's pool
        # captured on torch's side stream (it synchronises the device once, here); replays run on the
        # caller's current stream
        from .trainconv import hip_block_convs

        with torch.cuda.graph(g), hip_block_convs(self.network, self.hip_convs):
            with torch.autocast("cuda", dtype=torch.float16, enabled=self.autocast, cache_enabled=False):
                loss = az_loss(self.network, *self._g_in, self.q_average)
            loss.backward()
            self.optim.step()
        self.network.eval()
        self._g, self._g_loss = g, loss
        self.graph_captures += 1

    def train_batch(self, s, z, pi, q):
        """loss (mcts.py:234-252, via mcts.az_loss) -> zero_grad -> backward -> SGD step, with the
        network in train mode as the UpdateWorker runs it (updateworker.py:63); pinned by G8."""
        return float(self._train_step(s, z, pi, q))

    def lr_step(self, reward):
        self.scheduler.step(reward)
