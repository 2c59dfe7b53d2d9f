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

Evaluation games (SelfPlayWorker.set_up_policies(evaluate=True),
selfplayworker.py:68-94; compare_models, self_play_parallel.py:355-379): pass
`opponent=` a second network (its trees' leaves go to a second row segment
evaluated by that network), or "random" / "lookahead" for the hard-coded
players of games/general/hardcoded_players.py, optionally with its own
`opponent_iterations`; `record=False` skips Move records (update=False).
"""
import contextlib
import os
import time

import torch

from . import _lib, distributed
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

    def intervals(self, ref):
        """[(start_ms, end_ms)] of every recorded pair relative to the event `ref` (any stream)."""
        torch.cuda.synchronize()
        return [(ref.elapsed_time(a), ref.elapsed_time(b)) for a, b in self.pairs if b is not None]


def union_ms(intervals):
    """Length of the union of [start, end) intervals (ms): busy time of possibly overlapping launches."""
    total, cur_s, cur_e = 0.0, None, None
    for a, b in sorted(intervals):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        total += cur_e - cur_s
    return total


class SelfPlayEngine:
    def __init__(self, game, network, n_games=4096, iterations=200, alpha=1.0, strong_play=False, evaluate=False,
                 seed=0, subsequence0=None, rng="philox", max_games=None, device=None, dtype=torch.float16,
                 leaf_layout="nhwc", cpuct=4.0, x_noise=0.25, blocks_per_tree=0, bucket=256, opponent=None,
                 opponent_iterations=None, record=True, search_threads=1, leaf_dedup=None, opponent_alpha=None,
                 opponent_strong_play=None, opponent_search_threads=None, eval_cache=None):
        """opponent_alpha / opponent_strong_play / opponent_search_threads: the opposing MCTS side's own
        search settings (evaluation games: each side is built from its own container's kwargs,
        selfplayworker.py:71-81); None = the policy's.  dtype: the fused trunk's element type, fp16 by
        default (the reference's inference autocast, inference_worker.py:114-119) or bf16.  eval_cache: plies
        a position's network outputs stay cached (include/spmcts.h spmcts_set_eval_cache; 0 = off, 1 = within
        the ply that evaluated them); needs leaf dedup (pure evaluators, search_threads > 1); None = 1 where
        that holds, else 0."""
        self.game = game
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.evaluator = make_evaluator(network, game, device=self.device, dtype=dtype, leaf_layout=leaf_layout)
        # the opposing player: self-play (same network), a second network, or a hard-coded player
        self.evaluator1 = None
        opp_kind = _lib.PLAYER_MCTS
        if isinstance(opponent, str):
            kinds = {"random": _lib.PLAYER_RANDOM, "lookahead": _lib.PLAYER_LOOKAHEAD,
                     "onesteplookahead": _lib.PLAYER_LOOKAHEAD}
            if opponent.lower() not in kinds:
                raise ValueError(f"unknown hard-coded opponent {opponent!r} (random / lookahead)")
            opp_kind = kinds[opponent.lower()]
        elif opponent is not None and opponent is not network:
            self.evaluator1 = make_evaluator(opponent, game, device=self.device, dtype=dtype, leaf_layout=leaf_layout)
            e0, e1 = self.evaluator, self.evaluator1
            if (e0.leaf_format, e0.leaf_layout) != (e1.leaf_format, e1.leaf_layout):
                raise ValueError("both networks of an evaluation arena must take the same leaf format "
                                 f"({e0.leaf_format}/{e0.leaf_layout} vs {e1.leaf_format}/{e1.leaf_layout})")
        it1 = iterations if opponent_iterations is None else int(opponent_iterations)
        self.iterations = max(iterations, it1) if opp_kind == _lib.PLAYER_MCTS else iterations
        k0 = max(1, int(search_threads))
        k1 = k0 if opponent_search_threads is None or opp_kind != _lib.PLAYER_MCTS else max(1, int(opponent_search_threads))
        a1 = alpha if opponent_alpha is None else float(opponent_alpha)
        s1 = strong_play if opponent_strong_play is None else bool(opponent_strong_play)
        rank = distributed.env_rank()[0]
        if subsequence0 is None:
            subsequence0 = rank * 2 * n_games  # disjoint Philox subsequences per rank
        self.arena = Arena(game, n_trees=2 * n_games, n_games=n_games, iterations=self.iterations, rng=rng,
                           seed=seed, subsequence0=subsequence0, strong_play=strong_play, evaluate=evaluate,
                           leaf_format=self.evaluator.leaf_format, leaf_layout=self.evaluator.leaf_layout,
                           cpuct=cpuct, x_noise=x_noise, alpha=alpha, blocks_per_tree=blocks_per_tree,
                           device=self.device, search_threads=max(k0, k1))
        # K sims in flight per tree (the reference's thread_count search, mcts.py:328-331); a search of
        # `budget` sims with k in flight takes ceil(budget / k) network steps
        self.search_threads = self.arena.search_threads
        self.select_steps = -(-iterations // k0)
        if opp_kind == _lib.PLAYER_MCTS:
            self.select_steps = max(self.select_steps, -(-it1 // k1))
        if (k1, a1, s1) != (k0, alpha, strong_play) or k0 != self.search_threads:
            # tree 2g = the policy, 2g + 1 = the opposing player, each with its own kwargs
            self.arena.set_tree_search(alpha=[alpha, a1] * n_games, strong_play=[strong_play, s1] * n_games,
                                       search_threads=[k0, k1] * n_games)
        if self.evaluator1 is not None or opp_kind != _lib.PLAYER_MCTS or it1 != iterations:
            # tree 2g = the policy, 2g + 1 = the opposing player (selfplayworker.py:164-176)
            self.arena.set_tree_players(nets=[0, 1 if self.evaluator1 is not None else 0] * n_games,
                                        kinds=[_lib.PLAYER_MCTS, opp_kind] * n_games,
                                        budgets=[iterations, it1] * n_games)
        if not record:
            self.arena.games_set_record(False)
        # batch leaf dedup (include/spmcts.h spmcts_set_leaf_dedup): one row per distinct position of a
        # simulation step; by default on when every evaluator is a pure, batch-independent function of
        # the leaf planes (the fused HIP trunk), so each leaf still gets exactly its own outputs
        pure = all(getattr(ev, "pure_planes", False) for ev in (self.evaluator, self.evaluator1) if ev is not None)
        if leaf_dedup and not pure:
            # an evaluator whose outputs depend on the batch or the row (the torch TowerEvaluator's
            # batch-shaped heads, the per-row salted table net) would hand a duplicate its owner's outputs
            raise ValueError("leaf_dedup=True needs evaluators that are pure functions of the leaf planes "
                             "(pure_planes); leave it None to enable it only where that holds")
        self.leaf_dedup = bool(pure if leaf_dedup is None else leaf_dedup) and self.search_threads > 1
        if self.leaf_dedup:
            self.arena.set_leaf_dedup(True)
        # evaluation cache (include/spmcts.h spmcts_set_eval_cache): the dedup key extended over plies
        cache_ok = self.leaf_dedup  # pure evaluators (both networks of an evaluation arena: keys carry the network)
        self.eval_cache = (1 if cache_ok else 0) if eval_cache is None else int(eval_cache)
        if self.eval_cache and not cache_ok:
            raise ValueError("eval_cache needs leaf dedup (pure evaluators, search_threads > 1)")
        if self.eval_cache:
            self.arena.set_eval_cache(self.eval_cache)
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
        self.expand_timer = None
        self.nn_timer = None
        self.async_device = True  # device-count evaluators run a whole ply without host syncs
        for ev in (self.evaluator, self.evaluator1):  # outputs sized for every row the arena can emit
            if ev is not None and hasattr(ev, "reserve"):
                ev.reserve(self.arena.max_rows, self.device)
        self.refresh_root_prior()

    @torch.no_grad()
    def refresh_root_prior(self):
        """MCTreeSearch.reset evaluates the empty board (mcts.py:167-168); constant per weights."""
        a = self.arena
        for net, ev in enumerate((self.evaluator, self.evaluator1)):
            if ev is None:
                continue
            x = ev.empty_root_input(a.W, a.H, a.device)
            probs, _ = ev(x)
            a.set_root_prior(probs[0], net=net)

    def refresh_network(self):
        for ev in (self.evaluator, self.evaluator1):
            if ev is not None and hasattr(ev, "refresh"):
                ev.refresh()
        if self.eval_cache:
            self.arena.eval_cache_clear()  # outputs of the old weights leave the cache
        self.refresh_root_prior()

    def enable_timers(self, on=True):
        self.select_timer = EventTimer() if on else None
        self.expand_timer = EventTimer() if on else None
        self.nn_timer = EventTimer() if on else None
        self.tower_timer = EventTimer() if on else None
        for ev in (self.evaluator, self.evaluator1):
            if ev is not None:
                ev.tower_timer = self.tower_timer

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
        if self.evaluator1 is not None:
            return self._eval_expand2()
        m = min(a.max_rows, -(-n // self.bucket) * self.bucket)
        if self.nn_timer is not None:
            self.nn_timer.start()
        probs, values = self.evaluator(a.leaves(m))
        if self.nn_timer is not None:
            self.nn_timer.stop()
        a.expand(probs[:n], values[:n])
        self.nn_rows += n
        self.nn_rows_padded += m

    def _eval_expand2(self):
        """Two networks: rows [0, n0) through the policy's, rows [seg1, seg1 + n1) through the opponent's."""
        a = self.arena
        n0, n1 = a.segment_counts()
        outs = []
        for ev, row0, n, cap in ((self.evaluator, 0, n0, a.seg1), (self.evaluator1, a.seg1, n1, a.max_rows - a.seg1)):
            if n == 0:
                outs.append((self._dummy_out(), torch.zeros(1, device=a.device)))
                continue
            m = min(cap, -(-n // self.bucket) * self.bucket)
            if self.nn_timer is not None:
                self.nn_timer.start()
            outs.append(ev(a.leaves_from(row0, m)))
            if self.nn_timer is not None:
                self.nn_timer.stop()
            self.nn_rows += n
            self.nn_rows_padded += m
        (p0, v0), (p1, v1) = outs
        a.expand2(p0, v0, p1, v1)

    def _dummy_out(self):
        return torch.zeros((1, self.arena.A), dtype=torch.float32, device=self.arena.device)

    def _eval_expand_dev(self, cap=None, sim=False):
        """Network + expand on the device-side row count: no host synchronisation.  `cap` bounds the
        rows (and so the grid): a search step has at most one leaf per game, the end-of-ply
        expansions up to two.  `sim`: a simulation step, where a follower lane (LanedEngine cross-lane
        dedup) takes the rows its leader evaluated (Arena.peer_push)."""
        self._eval_dev(cap)
        self._expand_dev(sim)

    def _eval_dev(self, cap=None):
        """The network half of _eval_expand_dev (outputs kept for _expand_dev)."""
        a = self.arena
        if self.nn_timer is not None:
            self.nn_timer.start()
        if self.evaluator1 is None:
            rows = a.max_rows if cap is None else min(a.max_rows, cap)
            probs, values = self.evaluator.forward_dev(a.leaves(rows), a.count_dev, rows)
        else:
            probs, values = self.evaluator.forward_dev(a.leaves(a.seg1), a.segment_count_dev(0), a.seg1)
            cap1 = a.max_rows - a.seg1
            p1, v1 = self.evaluator1.forward_dev(a.leaves_from(a.seg1, cap1), a.segment_count_dev(1), cap1)
        if self.nn_timer is not None:
            self.nn_timer.stop()
        self._out = (probs, values) if self.evaluator1 is None else (probs, values, p1, v1)

    def _peer_push(self, sim=True):
        """A follower lane's simulation step: the leader's rows into ours (include/spmcts.h spmcts_peer_push: on the
        follower's push stream, once the leader's heads and our rows are done), outside the expand timer."""
        leader = getattr(self, "_leader", None)
        if leader is not None and sim and not getattr(self, "_pushed", False):
            _, lp, lv = leader.evaluator._dev_bufs
            self.arena.peer_push(self._out[0], self._out[1], lp, lv, self._leader_stream)
            self._pushed = True

    def _expand_dev(self, sim=False):
        """The expand half of _eval_expand_dev."""
        a = self.arena
        self._peer_push(sim)
        self._pushed = False
        if self.evaluator1 is None:
            probs, values = self._out
        else:
            probs, values, p1, v1 = self._out
        if self.expand_timer is not None:
            self.expand_timer.start()
        if self.evaluator1 is None:
            a.expand(probs, values)
        else:
            a.expand2(probs, values, p1, v1)
        if self.expand_timer is not None:
            self.expand_timer.stop()

    # --- one ply in phases (LanedEngine interleaves the phases of several engines on their streams)
    def _ply_begin(self):
        if not self.started:
            self.start()
        self.arena.games_begin_ply()

    def _ply_simulation(self, step=0):
        """One simulation step of every searching tree, without a host synchronisation.  With K > 1
        sims in flight only the first step launches the select kernel (it fills the K slots); later
        steps' selects run inside the expand kernel, which refills each slot right after its backup
        (the rolling schedule, csrc/spmcts.hip), so they only gather the pending leaves into rows."""
        self._ply_sim_net(step)
        self._expand_dev(sim=True)

    def _ply_sim_net(self, step=0):
        """The rows and network half of _ply_simulation."""
        if step == 0 or self.search_threads == 1:
            self.arena.select_async(self.select_timer)
        else:
            self.arena.leaf_rows_async()
        self._eval_dev(cap=self.n_games * self.search_threads)

    def _ply_move(self):
        self.arena.games_end_ply_async()
        self._eval_expand_dev(cap=2 * self.n_games)

    def ply(self, on_moves=None, refill=True, game_offset=0):
        """Advance every active game by one move. Returns (#games finished, #records exported).
        `game_offset` is added to the exported game ids (LanedEngine lanes)."""
        self._ply_begin()
        a = self.arena
        if self._device_count_ok():
            for i in range(self.select_steps):
                self._ply_simulation(i)
            self._ply_move()
        else:
            for _ in range(self.select_steps):
                self._eval_expand(a.select(self.select_timer))
            self._eval_expand(a.games_end_ply())
        return self._ply_finish(on_moves, refill, game_offset)

    def _ply_finish(self, on_moves=None, refill=True, game_offset=0):
        return self._ply_finish_result(self._ply_finish_async(refill), on_moves, game_offset)

    def _ply_finish_async(self, refill=True):
        """The ply's results and Move export queued on the current stream (Arena.finish_export_async)."""
        return self.arena.finish_export_async(refill=refill)

    def _ply_finish_result(self, ev, on_moves=None, game_offset=0):
        """Wait for _ply_finish_async's event, hand the Moves on, count them."""
        finished, moves = self.arena.finish_export_result(ev)
        exported = 0
        if moves is not None:
            if game_offset:
                moves["game"] += game_offset
            exported = int(moves["z"].shape[0])
            if on_moves is not None:
                on_moves(moves)
        self.games_done += finished
        self.positions += exported
        self.plies += 1
        return finished, exported

    def _device_count_ok(self):
        return self.async_device and all(getattr(ev, "supports_device_count", False)
                                         for ev in (self.evaluator, self.evaluator1) if ev is not None)

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

    def play_games(self, n, on_moves=None, on_ply=None, exchange=None, every=8):
        """Play exactly `n` more games (refilling slots on device until n have started).

        Returns the number of plies it took.  Game ids continue from earlier calls, so
        swap_sides alternates across calls exactly as the reference's task ids do.
        Finished games' Move records reach `on_moves` through a distributed.MoveExchange: at once
        in a single process; under torch.distributed batched to rank 0 every `every` plies (the
        episode-batch exchange), where every rank plays its own `n` and keeps stepping idle plies
        until an exchange round finds all ranks done, so the collectives stay matched."""
        target = self._play_games_setup(n)
        if n <= 0 and not distributed.is_distributed():
            return 0
        ex = exchange if exchange is not None else distributed.MoveExchange(*self._record_shape(), sink=on_moves,
                                                                            every=every)
        plies = 0
        while True:
            self.ply(on_moves=ex.stage)
            plies += 1
            if on_ply is not None:
                on_ply(self)
            # the statistics are read (a host sync on the device counters) only for a real exchange round
            r = ex.end_ply(self.stats_vector if distributed.is_distributed() else None, done=self.games_done >= target)
            if r is not None and r[0]:
                break
        self._started = self._limit
        return plies

    def _record_shape(self):
        return self.arena.cells, self.arena.A

    def _play_games_setup(self, n):
        """Raise the game budget by `n` and start idle slots; returns the games_done target."""
        a = self.arena
        started = getattr(self, "_started", 0)
        limit = started + max(0, n)
        if n > 0:
            a.games_set_limit(limit)
            st = a.games_state()
            idle = [i for i, s in enumerate(st["state"]) if s == 0]
            k = min(len(idle), n)
            if k:
                a.games_start(idle[:k])
            self.started = True
        self._limit = limit
        return self.games_done + max(0, n)

    def counters(self):
        return self.arena.counters()

    @property
    def weights_snapshot(self):
        """True when every leaf evaluator reads its own copy of the weights (Evaluator.snapshot), so
        SGD steps may run on another stream beside this engine's plies."""
        return all(getattr(ev, "snapshot", False) for ev in (self.evaluator, self.evaluator1) if ev is not None)

    def stats_vector(self):
        """[games, moves, first w/d/l, second w/d/l] for the episode-end all_reduce."""
        c = self.arena.counters()
        r = c["results"]
        return [c["games_finished"], c["moves"], r[0][0], r[0][1], r[0][2], r[1][0], r[1][1], r[1][2]]

    def check(self):
        self.arena.check()


class _SumTimer:
    """The per-lane EventTimers of one kind seen as one (sums; launches of all lanes)."""

    def __init__(self, timers):
        self.timers = timers

    def total_ms(self):
        return sum(t.total_ms() for t in self.timers)

    def count(self):
        return sum(t.count() for t in self.timers)

    def intervals(self, ref):
        return [iv for t in self.timers for iv in t.intervals(ref)]


class LanedEngine:
    """`lanes` SelfPlayEngines of n_games / lanes slots each, on their own HIP streams, stepped in
    lock step: every simulation issues each lane's select -> tower -> heads -> expand on that lane's
    stream, so one lane's tree kernels (and the tail workgroups of its tower launch) run beside the
    other lane's tower launch instead of leaving the chip idle between dependent launches.

    Same public surface as SelfPlayEngine (ply / run / play_games / counters / stats_vector / check /
    enable_timers / refresh_network).  Lane i uses the Philox subsequences of trees
    [offset_i, offset_i + 2 n_i) of a single arena of n_games slots (same seed), and its exported
    game ids are offset by i * 2**40 (even, so swap_sides = id odd is preserved and ids stay unique).
    Each lane is a complete arena: results are those of `lanes` independent engines.  With `pack`
    the fused tower packs every lane's batch into full tiles (SPMCTS_TOWER_PACK) rather than whole
    chip rounds, since the lanes' concurrent launches fill each other's partial rounds.

    `stagger` (off by default; device-count evaluators): lane i runs i * S / lanes simulation steps behind
    lane 0 (S = simulation steps per ply), so the lanes' ply boundaries -- the host round trips of
    the move export and the first fill of the next searches (k_select_vl), whose slowest trees run
    long serial chains of terminal simulations -- fall under another lane's tower launches instead of
    coinciding.  Every lane still runs begin -> S steps -> move -> finish per ply on its own stream
    (the same work in the same order: per-lane results are unchanged); only the interleaving of the
    lanes changes.  A ply() call finishes one ply of every lane (lane i > 0: the one it began in the
    previous call; on the first call it only begins one); `drain()` completes the plies staggered lanes
    have in flight (run() and play_games() end with it, so they return at ply boundaries as before).
    Measured on one box (profiles/r04/stagger/): ply-start tower-free time 1.6 % -> 0.8 % of a
    steady-state ply, steady-state positions/s +0.4 %, the driver's short run -0.6 %: off by default."""

    GAME_ID_STRIDE = 1 << 40

    def __init__(self, game, network, n_games=4096, lanes=2, seed=0, subsequence0=None, device=None, pack=True,
                 stagger=False, cross_dedup=None, lane_sizes=None, **kw):
        if lanes < 1 or n_games < lanes:
            raise ValueError(f"need 1 <= lanes <= n_games (lanes={lanes}, n_games={n_games})")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        rank = distributed.env_rank()[0]
        if subsequence0 is None:
            subsequence0 = rank * 2 * n_games
        sizes = [n_games // lanes + (1 if i < n_games % lanes else 0) for i in range(lanes)]
        if lane_sizes is not None:  # an explicit split of the n_games slots over the lanes
            sizes = [int(x) for x in lane_sizes]
            if len(sizes) != lanes or sum(sizes) != n_games or min(sizes) < 1:
                raise ValueError(f"lane_sizes {lane_sizes} must be {lanes} positive counts summing to {n_games}")
        # a game budget is split like the slots (each lane stops starting games at its share)
        self.max_games = kw.pop("max_games", None)
        budgets = [None] * lanes if self.max_games is None else \
            [self.max_games // lanes + (1 if i < self.max_games % lanes else 0) for i in range(lanes)]
        # SPMCTS_LANE_PRIORITY=1: lane 0's stream at high priority, so its tower workgroups are dispatched
        # first and the lanes' tree phases fall under each other's towers instead of coinciding
        prio = os.environ.get("SPMCTS_LANE_PRIORITY", "0") == "1"
        self.streams = [torch.cuda.Stream(device=self.device, priority=(-1 if prio and i == 0 else 0))
                        for i in range(lanes)]
        self.lanes = []
        off = 0
        for i, (n, st) in enumerate(zip(sizes, self.streams)):
            with torch.cuda.stream(st):
                self.lanes.append(SelfPlayEngine(game, network, n_games=n, seed=seed, subsequence0=subsequence0 + 2 * off,
                                                 device=self.device, max_games=budgets[i], **kw))
            off += n
        torch.cuda.synchronize(self.device)
        if lanes > 1 and pack:
            for e in self.lanes:  # tower launches share the chip: full tiles, no round alignment
                for ev in (e.evaluator, e.evaluator1):
                    if ev is not None and hasattr(ev, "concurrent"):
                        ev.concurrent = True
        self.n_games = n_games
        self.stagger = bool(stagger) and lanes > 1
        self._pending = False  # staggered lanes i > 0 are part-way through a ply
        # cross-lane leaf dedup (round 6, include/spmcts.h spmcts_set_leaf_peer): lanes i > 0 follow lane 0 --
        # a pending leaf whose network input lane 0 evaluates in the same simulation step takes lane 0's row.
        # Needs lanes in lock step (no stagger), leaf dedup (pure, batch-independent evaluators) and
        # single-network arenas; default on where those hold.  Results are unchanged bit for bit
        # (tests/test_gpu_engine.py), only the rows evaluated drop.
        e0 = self.lanes[0]
        ok = (lanes > 1 and not self.stagger and e0.leaf_dedup and all(e.evaluator1 is None for e in self.lanes)
              and all(e.arena.seg1 >= e.arena.n_trees * e.search_threads for e in self.lanes)
              and all(e._device_count_ok() for e in self.lanes))
        if cross_dedup and not ok:
            raise ValueError("cross_dedup needs lanes > 1 in lock step, leaf dedup and single-network device-count "
                             "evaluators")
        self.cross_dedup = bool(ok if cross_dedup is None else cross_dedup)
        if self.cross_dedup:
            for e in self.lanes[1:]:
                e.arena.set_leaf_peer(e0.arena)
                e._leader, e._leader_stream = e0, self.streams[0]
        self.iterations = self.lanes[0].iterations
        self.select_steps = self.lanes[0].select_steps
        self.search_threads = self.lanes[0].search_threads
        self.leaf_dedup = self.lanes[0].leaf_dedup
        self.eval_cache = self.lanes[0].eval_cache
        self.evaluator = self.lanes[0].evaluator
        self.select_timer = self.expand_timer = self.nn_timer = self.tower_timer = None

    def _each(self, fn):
        out = []
        for e, st in zip(self.lanes, self.streams):
            with torch.cuda.stream(st):
                out.append(fn(e))
        return out

    def _lanes_wait_caller(self):
        """Order the lanes' next work after everything the caller queued on its own stream (trainer
        steps reading the replay ring the lanes append to, optimizer updates of the weights that
        refresh_network packs): the lanes never run ahead of the caller's stream."""
        for st in self.streams:
            if st is not None:
                st.wait_stream(torch.cuda.current_stream(self.device))

    @property
    def positions(self):
        return sum(e.positions for e in self.lanes)

    @property
    def games_done(self):
        return sum(e.games_done for e in self.lanes)

    @property
    def started(self):
        return all(e.started for e in self.lanes)

    def start(self):
        self._each(lambda e: e.start())

    def enable_timers(self, on=True):
        self._each(lambda e: e.enable_timers(on))
        if on:
            self.select_timer = _SumTimer([e.select_timer for e in self.lanes])
            self.expand_timer = _SumTimer([e.expand_timer for e in self.lanes])
            self.nn_timer = _SumTimer([e.nn_timer for e in self.lanes])
            self.tower_timer = _SumTimer([e.tower_timer for e in self.lanes])
        else:
            self.select_timer = self.expand_timer = self.nn_timer = self.tower_timer = None

    def refresh_network(self, on_moves=None):
        """New weights for every lane.  A staggered lane may hold a half-finished ply (between ply()
        calls): it is finished on the old weights first (drain, its Moves to `on_moves`), so no search
        mixes evaluations of two weight versions; without `on_moves` that would drop its finished games'
        Moves, so it raises instead (run() and play_games() return drained)."""
        if getattr(self, "_pending", False):
            if on_moves is None:
                raise RuntimeError("refresh_network with a staggered ply in flight: pass on_moves (or call "
                                   "drain(on_moves) first) so the games it finishes are not dropped")
            self.drain(on_moves)
        self._lanes_wait_caller()
        self._each(lambda e: e.refresh_network())

    def _stream(self, st):
        return torch.cuda.stream(st) if st is not None else contextlib.nullcontext()

    def _lags(self):
        """Simulation steps lane i runs behind lane 0 when staggered."""
        S, L = self.select_steps, len(self.lanes)
        return [i * S // L for i in range(L)]

    def _staggered(self):
        return (getattr(self, "stagger", False) and 1 < len(self.lanes) <= self.select_steps
                and all(e._device_count_ok() for e in self.lanes))

    def _ply_staggered(self, on_moves, refill):
        """One ply of every lane, lane i lag[i] steps behind lane 0.  Issue order (each stream keeps its
        own op order, so per-lane results are unchanged): lane 0's whole ply up to its move, interleaved
        with the last lag[i] steps of the ply lane i > 0 began in the previous call; then lane i's move
        and finish (the host reads its counts while lane 0's queued half ply keeps the chip busy) and
        the first S - lag[i] steps of its next ply; then lane 0's finish (lane i's queued steps keep the
        chip busy).  On the first call (nothing in flight) lane i > 0 only begins its ply."""
        S, lag = self.select_steps, self._lags()
        lanes, streams = self.lanes, self.streams
        pending = getattr(self, "_pending", False)
        res = [(0, 0)] * len(lanes)
        with self._stream(streams[0]):
            lanes[0]._ply_begin()
        for t in range(S):
            for i, (e, st) in enumerate(zip(lanes, streams)):
                with self._stream(st):
                    if i == 0:
                        e._ply_simulation(t)
                    elif pending and t < lag[i]:  # the ply begun in the previous call
                        e._ply_simulation(S - lag[i] + t)
        with self._stream(streams[0]):
            lanes[0]._ply_move()
        for i in range(1, len(lanes)):
            e = lanes[i]
            with self._stream(streams[i]):
                if pending:
                    e._ply_move()
                    res[i] = e._ply_finish(on_moves, refill, game_offset=i * self.GAME_ID_STRIDE)
                e._ply_begin()
                for s in range(S - lag[i]):
                    e._ply_simulation(s)
        with self._stream(streams[0]):
            res[0] = lanes[0]._ply_finish(on_moves, refill, game_offset=0)
        self._pending = True
        return res

    def drain(self, on_moves=None, refill=True):
        """Complete the plies that staggered lanes have in flight, so every lane stands at a ply boundary.
        Returns (#games finished, #records exported) of those plies."""
        if not getattr(self, "_pending", False):
            return 0, 0
        S, lag = self.select_steps, self._lags()
        res = []
        for i in range(1, len(self.lanes)):
            e, st = self.lanes[i], self.streams[i]
            with self._stream(st):
                for s in range(S - lag[i], S):
                    e._ply_simulation(s)
                e._ply_move()
                res.append(e._ply_finish(on_moves, refill, game_offset=i * self.GAME_ID_STRIDE))
        self._pending = False
        self._caller_waits_lanes()
        return sum(r[0] for r in res), sum(r[1] for r in res)

    def _caller_waits_lanes(self):
        for st in self.streams:  # later work on the caller's stream sees every lane's work
            if st is not None:
                torch.cuda.current_stream(self.device).wait_stream(st)

    def ply(self, on_moves=None, refill=True):
        """One move of every active game of every lane. Returns (#games finished, #records exported)."""
        self._lanes_wait_caller()
        if self._staggered():
            res = self._ply_staggered(on_moves, refill)
        elif not all(e._device_count_ok() for e in self.lanes):  # host-synchronised evaluators: lane by lane
            res = []
            for i, (e, st) in enumerate(zip(self.lanes, self.streams)):
                with self._stream(st):
                    res.append(e.ply(on_moves, refill, game_offset=i * self.GAME_ID_STRIDE))
        else:
            self._each(lambda e: e._ply_begin())
            for i in range(self.select_steps):
                # every lane's rows and network first, then the followers' leader-served rows (issued once lane 0's
                # heads are queued: spmcts_peer_push), then the expands; per stream the order is one lane's ply
                self._each(lambda e: e._ply_sim_net(i))
                self._each(lambda e: e._peer_push())
                self._each(lambda e: e._expand_dev(sim=True))
            self._each(lambda e: e._ply_move())
            # every lane's results and export queued before the host waits on any of them (one round trip)
            evs = self._each(lambda e: e._ply_finish_async(refill))
            res = []
            for i, (e, st, ev) in enumerate(zip(self.lanes, self.streams, evs)):
                with self._stream(st):  # on_moves runs on the lane's stream, after its export
                    res.append(e._ply_finish_result(ev, on_moves, game_offset=i * self.GAME_ID_STRIDE))
        self._caller_waits_lanes()
        return sum(r[0] for r in res), sum(r[1] for r in res)

    def run(self, plies=None, games=None, seconds=None, on_moves=None):
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
        self.drain(on_moves=on_moves)  # staggered lanes finish the ply they have in flight
        return dict(plies=n, seconds=time.time() - t0, games=self.games_done, positions=self.positions)

    def play_games(self, n, on_moves=None, on_ply=None, exchange=None, every=8):
        """As SelfPlayEngine.play_games, the n games split over the lanes (one exchange for all lanes).
        Staggered lanes start and end at ply boundaries: a ply a lane has in flight is completed first
        (its records go into this call's exchange), and the ply each lane i > 0 has in flight when the
        last round finds every rank done is completed before returning, its records sent in one more
        (forced) exchange round, which every rank runs."""
        self._lanes_wait_caller()
        ex = exchange if exchange is not None else distributed.MoveExchange(*self.lanes[0]._record_shape(),
                                                                            sink=on_moves, every=every)
        self.drain(on_moves=ex.stage)
        k = len(self.lanes)
        parts = [n // k + (1 if i < n % k else 0) for i in range(k)]
        targets = []
        for e, st, m in zip(self.lanes, self.streams, parts):
            with torch.cuda.stream(st):
                targets.append(e._play_games_setup(m))
        if n <= 0 and not distributed.is_distributed():
            return 0
        plies = 0
        while True:
            self.ply(on_moves=ex.stage)
            plies += 1
            if on_ply is not None:
                on_ply(self)
            r = ex.end_ply(self.stats_vector if distributed.is_distributed() else None,
                           done=all(e.games_done >= t for e, t in zip(self.lanes, targets)))
            if r is not None and r[0]:
                break
        if getattr(self, "_pending", False):
            self.drain(on_moves=ex.stage)
            if distributed.is_distributed():  # every rank ended on the same round: one more, together
                ex.end_ply(self.stats_vector, done=True, force=True)
        for e in self.lanes:
            e._started = e._limit
        return plies

    @property
    def weights_snapshot(self):
        return all(e.weights_snapshot for e in self.lanes)

    def counters(self):
        cs = self._each(lambda e: e.counters())
        out = {}
        for k, v in cs[0].items():
            if k == "results":
                out[k] = [[sum(c[k][i][j] for c in cs) for j in range(3)] for i in range(2)]
            elif k == "blocks_in_use_max":
                out[k] = max(c[k] for c in cs)
            elif k == "error_flags":
                out[k] = 0
                for c in cs:
                    out[k] |= c[k]
            else:
                out[k] = sum(c[k] for c in cs)
        return out

    def stats_vector(self):
        vs = self._each(lambda e: e.stats_vector())
        return [sum(x) for x in zip(*vs)]

    def check(self):
        self._each(lambda e: e.check())
