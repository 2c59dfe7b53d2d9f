"""Batched self-play engine: thousands of SelfPlayer episodes in lock step on one GPU.

Replaces the SelfPlayWorker processes x game threads x search threads of the
reference (games/algos/self_play_parallel.py:95-171, selfplayworker.py:95-224)
with one arena of `n_games` game slots (two trees each).  One *ply* advances
every active game by one move:

    games_begin_ply                  Dirichlet noise on each mover's root
    iterations x (select -> network -> expand)      search_node for every game
    games_end_ply -> network -> expand              _play + env.step + play_action
    games_finish_ply                 results, Move export, slot refill

Finished games export their Move records (policy's then opponent's, with
actual_val = the owner's result, mcts.py:225-232) and the slot is refilled
with the next game id (swap_sides = id odd, self_play_parallel.py:237) until
`max_games` games have been started.

Network batches are padded up to a multiple of `bucket` rows (stale rows are
evaluated and ignored), so the convolution library sees a handful of shapes
instead of one per simulation.
"""
import time

import torch

from . import distributed
from .arena import Arena
from .evaluator import make_evaluator


class EventTimer:
    """Accumulates GPU time between start()/stop() pairs with HIP events on the current stream."""

    def __init__(self):
        self.pairs = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.pairs.append([e, None])

    def stop(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.pairs[-1][1] = e

    def reset(self):
        self.pairs = []

    def total_ms(self):
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.pairs if b is not None)

    def count(self):
        return len(self.pairs)


class SelfPlayEngine:
    def __init__(self, game, network, n_games=4096, iterations=200, alpha=1.0, strong_play=False, evaluate=False,
                 seed=0, subsequence0=None, rng="philox", max_games=None, device=None, dtype=torch.bfloat16,
                 leaf_layout="nhwc", cpuct=4.0, x_noise=0.25, blocks_per_tree=0, bucket=256):
        self.game = game
        self.iterations = iterations
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.evaluator = make_evaluator(network, game, device=self.device, dtype=dtype, leaf_layout=leaf_layout)
        rank = distributed.env_rank()[0]
        if subsequence0 is None:
            subsequence0 = rank * 2 * n_games  # disjoint Philox subsequences per rank
        self.arena = Arena(game, n_trees=2 * n_games, n_games=n_games, iterations=iterations, rng=rng, seed=seed,
                           subsequence0=subsequence0, strong_play=strong_play, evaluate=evaluate,
                           leaf_format=self.evaluator.leaf_format, leaf_layout=self.evaluator.leaf_layout,
                           cpuct=cpuct, x_noise=x_noise, alpha=alpha, blocks_per_tree=blocks_per_tree,
                           device=self.device)
        self.n_games = n_games
        self.max_games = max_games
        # torch convolutions want few distinct shapes; the fused HIP tower takes any batch
        self.bucket = max(1, int(getattr(self.evaluator, "bucket", bucket)))
        self.positions = 0
        self.games_done = 0
        self.nn_rows = 0
        self.nn_rows_padded = 0
        self.plies = 0
        self.started = False
        self.select_timer = None
        self.nn_timer = None
        self.async_device = True  # device-count evaluators run a whole ply without host syncs
        self.refresh_root_prior()

    @torch.no_grad()
    def refresh_root_prior(self):
        """MCTreeSearch.reset evaluates the empty board (mcts.py:167-168); constant per weights."""
        a = self.arena
        x = self.evaluator.empty_root_input(a.W, a.H, a.device)
        probs, _ = self.evaluator(x)
        a.set_root_prior(probs[0])

    def refresh_network(self):
        if hasattr(self.evaluator, "refresh"):
            self.evaluator.refresh()
        self.refresh_root_prior()

    def enable_timers(self, on=True):
        self.select_timer = EventTimer() if on else None
        self.nn_timer = EventTimer() if on else None
        self.tower_timer = EventTimer() if on else None
        self.evaluator.tower_timer = self.tower_timer

    def start(self):
        """Fill every slot and keep refilling (until `max_games` games have started, if set)."""
        a = self.arena
        first = self.n_games if self.max_games is None else min(self.n_games, self.max_games)
        a.games_set_limit(-1 if self.max_games is None else self.max_games)
        a.games_start(list(range(first)))
        self._started = first if self.max_games is None else self.max_games
        self.started = True

    def _eval_expand(self, n):
        if not n:
            return
        a = self.arena
        m = min(a.max_rows, -(-n // self.bucket) * self.bucket)
        if self.nn_timer is not None:
            self.nn_timer.start()
        probs, values = self.evaluator(a.leaves(m))
        if self.nn_timer is not None:
            self.nn_timer.stop()
        a.expand(probs[:n], values[:n])
        self.nn_rows += n
        self.nn_rows_padded += m

    def _eval_expand_dev(self):
        """Network + expand on the device-side row count: no host synchronisation."""
        a = self.arena
        if self.nn_timer is not None:
            self.nn_timer.start()
        probs, values = self.evaluator.forward_dev(a.leaves(a.max_rows), a.count_dev, a.max_rows)
        if self.nn_timer is not None:
            self.nn_timer.stop()
        a.expand(probs, values)

    def ply(self, on_moves=None, refill=True):
        """Advance every active game by one move. Returns (#games finished, #records exported)."""
        if not self.started:
            self.start()
        a = self.arena
        a.games_begin_ply()
        if getattr(self.evaluator, "supports_device_count", False) and self.async_device:
            for _ in range(self.iterations):
                a.select_async(self.select_timer)
                self._eval_expand_dev()
            a.games_end_ply_async()
            self._eval_expand_dev()
        else:
            for _ in range(self.iterations):
                self._eval_expand(a.select(self.select_timer))
            self._eval_expand(a.games_end_ply())
        finished, ring = a.games_finish_ply(refill=refill)
        exported = 0
        if ring:
            moves = a.export_moves(ring)
            exported = int(moves["z"].shape[0])
            if on_moves is not None:
                on_moves(moves)
        self.games_done += finished
        self.positions += exported
        self.plies += 1
        return finished, exported

    def run(self, plies=None, games=None, seconds=None, on_moves=None):
        """Play until `plies` plies / `games` finished games / `seconds` elapse / the game budget is spent."""
        t0 = time.time()
        n = 0
        while True:
            self.ply(on_moves=on_moves)
            n += 1
            if plies is not None and n >= plies:
                break
            if games is not None and self.games_done >= games:
                break
            if seconds is not None and time.time() - t0 >= seconds:
                break
            if self.max_games is not None and self.games_done >= self.max_games:
                break
        return dict(plies=n, seconds=time.time() - t0, games=self.games_done, positions=self.positions)

    def play_games(self, n, on_moves=None, on_ply=None):
        """Play exactly `n` more games (refilling slots on device until n have started).

        Returns the number of plies it took.  Game ids continue from earlier calls, so
        swap_sides alternates across calls exactly as the reference's task ids do."""
        a = self.arena
        if n <= 0:
            return 0
        started = getattr(self, "_started", 0)
        limit = started + n
        a.games_set_limit(limit)
        st = a.games_state()
        idle = [i for i, s in enumerate(st["state"]) if s == 0]
        k = min(len(idle), n)
        if k:
            a.games_start(idle[:k])
        self.started = True
        target = self.games_done + n
        plies = 0
        while self.games_done < target:
            self.ply(on_moves=on_moves)
            plies += 1
            if on_ply is not None:
                on_ply(self)
        self._started = limit
        return plies

    def counters(self):
        return self.arena.counters()

    def stats_vector(self):
        """[games, moves, first w/d/l, second w/d/l] for the episode-end all_reduce."""
        c = self.arena.counters()
        r = c["results"]
        return [c["games_finished"], c["moves"], r[0][0], r[0][1], r[0][2], r[1][0], r[1][1], r[1][2]]

    def check(self):
        self.arena.check()
