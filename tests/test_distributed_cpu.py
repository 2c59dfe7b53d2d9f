"""CPU: the multi-GPU exchange steps with torch.distributed gloo, world sizes 2, 4 and 8: the
episode-batch MoveExchange (Move rows staged per rank, one header all_gather + one gather to rank 0
per round, statistics summed in the same round), the engines' play_games loops that end on it,
the primitives (stats all_reduce, max, one-buffer weight broadcast), and the self-launch helpers that
start one process per GPU (bench.py --gpus N, SelfPlayScheduler(gpus=N))."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from self_play_reinforcement_learning_amd import distributed as D


def _free_port():
    """A rendezvous for one test: a fresh file store (SPMCTS_DIST_INIT), so concurrent or
    back-to-back tests never race for a TCP port."""
    return tempfile.mkdtemp(prefix="spmcts_dist_") + "/store"


def _by_value(obj):
    """Tensors -> numpy for a result queue: torch shares CPU tensors through file descriptors that the
    sending process must outlive, and the rank workers exit right after putting their results."""
    if isinstance(obj, torch.Tensor):
        return ("__t__", obj.detach().cpu().numpy())
    if isinstance(obj, dict):
        return {k: _by_value(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_by_value(v) for v in obj)
    return obj


def _restore(obj):
    if isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[0], str) and obj[0] == "__t__":
        return torch.from_numpy(obj[1])
    if isinstance(obj, dict):
        return {k: _restore(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_restore(v) for v in obj)
    return obj


def _moves(rank, n):
    g = torch.Generator().manual_seed(rank)
    return dict(
        state=torch.randint(-1, 2, (n, 42), dtype=torch.int8, generator=g),
        tree_probs=torch.rand(n, 7, generator=g),
        q=torch.rand(n, generator=g, dtype=torch.float64),
        q_f64=torch.randint(0, 2, (n,), dtype=torch.uint8, generator=g),
        z=torch.randint(-1, 2, (n,), generator=g).float(),
        game=torch.arange(n, dtype=torch.int64) + 1000 * rank,
    )


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      SPMCTS_DIST_INIT="file://" + port)
    D.init_from_env(backend="gloo")
    stats = D.all_reduce_stats([rank + 1, 10 * rank, 1, 0, 0, 0, 1, 0])
    mx = D.all_reduce_max(float(rank) * 1.5)
    net = torch.nn.Sequential(torch.nn.Linear(4, 2), torch.nn.BatchNorm1d(2))  # float + int64 state
    with torch.no_grad():
        net[0].weight.fill_(float(rank))
        net[1].running_mean.fill_(float(rank) + 0.5)
        net[1].num_batches_tracked.fill_(7 + rank)
    D.broadcast_state_dict(net)
    sd = net.state_dict()
    q.put(_by_value((rank, stats.tolist(), None, mx, float(net[0].weight.sum()),
                     [float(sd["1.running_mean"].sum()), int(sd["1.num_batches_tracked"])])))
    torch.distributed.destroy_process_group()


class _FakeArena:
    def __init__(self, slots):
        self.slots = slots

    def games_set_limit(self, n):
        self.limit = n

    def games_state(self):
        import numpy as np

        return {"state": np.zeros(self.slots, dtype=int)}

    def games_start(self, slots):
        self.started = list(slots)


class _FakeEngine:
    """Stands in for SelfPlayEngine inside its own play_games loop: rank r finishes r + 1 games per
    ply (while it has games left) and exports one Move record per finished game."""

    def __init__(self, rate, rank=0):
        self.arena = _FakeArena(4)
        self.games_done = 0
        self.rate = rate
        self.rank = rank
        self.plies_run = 0
        self._limit = 0

    def ply(self, on_moves=None):
        self.plies_run += 1
        k = max(0, min(self.rate, self._limit - self.games_done))
        m = _moves(self.rank, k)
        m["game"] = torch.arange(self.games_done, self.games_done + k, dtype=torch.int64) + 1000 * self.rank
        self.games_done += k
        on_moves(m)

    def stats_vector(self):
        return [self.games_done, 0, 0, 0, 0, 0, 0, 0]

    def _record_shape(self):
        return 42, 7

    def _play_games_setup(self, n):
        from self_play_reinforcement_learning_amd.engine import SelfPlayEngine

        return SelfPlayEngine._play_games_setup(self, n)


def _loop_worker(rank, world, port, q):
    from self_play_reinforcement_learning_amd.engine import SelfPlayEngine

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      SPMCTS_DIST_INIT="file://" + port)
    D.init_from_env(backend="gloo")
    eng = _FakeEngine(rate=rank + 1, rank=rank)
    gathered = []
    plies = SelfPlayEngine.play_games(eng, 6, on_moves=lambda m: gathered.append(m["game"].tolist()), every=4)
    q.put(_by_value((rank, plies, eng.games_done, gathered)))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_play_games_keeps_ranks_in_step_gloo(world):
    """Ranks that finish their share early keep stepping idle plies until an exchange round finds
    every rank done (so the rounds always match, no deadlock); every finished game's records reach
    rank 0 exactly once, batched per round (every 4 plies), and no other rank's sink is called."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_restore(q.get(timeout=120)) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 0 (1 game per ply) needs 6 plies -> the round after ply 8 finds everyone done
    assert all(r[1] == 8 for r in res)
    assert all(r[2] == 6 for r in res)
    assert all(r[3] == [] for r in res[1:])
    rounds = res[0][3]
    assert len(rounds) == 2
    got = sorted(g for batch in rounds for g in batch)
    assert got == sorted(1000 * r + i for r in range(world) for i in range(6))
    # a round holds rank 0's rows first, then rank 1's, ...
    assert rounds[0][:4] == [0, 1, 2, 3] and rounds[0][4] == 1000


class _FakeLane(_FakeEngine):
    """A LanedEngine lane: the phase methods of SelfPlayEngine.ply; finishes `rate` games per ply."""

    iterations = 3
    select_steps = 3

    def _device_count_ok(self):
        return True

    def _ply_begin(self):
        self.sims = 0

    def _ply_simulation(self, step=0):
        self.sims += 1

    def _ply_sim_net(self, step=0):  # LanedEngine's lock-step split of _ply_simulation
        self.sims += 1

    def _peer_push(self, sim=True):
        pass

    def _expand_dev(self, sim=False):
        pass

    def _ply_move(self):
        assert self.sims == self.iterations

    def _ply_finish_async(self, refill=True):  # LanedEngine queues every lane's finish before reading any
        return ("finish", self.plies_run)

    def _ply_finish_result(self, ev, on_moves=None, game_offset=0):
        assert ev == ("finish", self.plies_run)
        return self._ply_finish(on_moves, game_offset=game_offset)

    def _ply_finish(self, on_moves=None, refill=True, game_offset=0):
        self.plies_run += 1
        k = max(0, min(self.rate, self._limit - self.games_done))
        m = _moves(self.rank, k)
        m["game"] = torch.arange(self.games_done, self.games_done + k, dtype=torch.int64) + 1000 * self.rank + game_offset
        self.games_done += k
        on_moves(m)
        return k, k


def _laned_worker(rank, world, port, q):
    from self_play_reinforcement_learning_amd.engine import LanedEngine

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      SPMCTS_DIST_INIT="file://" + port)
    D.init_from_env(backend="gloo")
    eng = LanedEngine.__new__(LanedEngine)  # lanes without a GPU: no streams, fake arenas
    eng.lanes = [_FakeLane(rate=rank + 1, rank=rank), _FakeLane(rate=1, rank=rank)]
    eng.streams = [None, None]
    eng.iterations = 3
    eng.select_steps = 3
    eng.device = torch.device("cpu")
    games = []
    plies = eng.play_games(8, on_moves=lambda m: games.extend(m["game"].tolist()), every=2)
    q.put(_by_value((rank, plies, [ln.games_done for ln in eng.lanes], games)))
    torch.distributed.destroy_process_group()


def test_laned_engine_play_games_gloo():
    """LanedEngine splits the games over its lanes, every lane steps every ply, both lanes' records
    go through one exchange, and lane i's game ids carry the i * 2**40 offset."""
    from self_play_reinforcement_learning_amd.engine import LanedEngine

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_laned_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([_restore(q.get(timeout=120)) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, d0, g0), (_, p1, d1, g1) = res
    # 8 games = 4 per lane; the slowest lane (rate 1) needs 4 plies, a round every 2 plies
    assert p0 == p1 == 4
    assert d0 == [4, 4] and d1 == [4, 4]
    assert g1 == []
    S = LanedEngine.GAME_ID_STRIDE
    assert sorted(g0) == sorted([i for i in range(4)] + [S + i for i in range(4)] +
                                [1000 + i for i in range(4)] + [S + 1000 + i for i in range(4)])


class _SeqLane(_FakeLane):
    """A _FakeLane that records its phase calls (and checks a ply's steps run in order)."""

    select_steps = 4
    iterations = 4

    def __init__(self, log, idx, **kw):
        super().__init__(**kw)
        self.log, self.idx = log, idx

    def _ply_begin(self):
        self.log.append((self.idx, "begin"))
        self.sims = 0

    def _ply_simulation(self, step=0):
        assert step == self.sims, (self.idx, step, self.sims)
        self.log.append((self.idx, step))
        self.sims += 1

    def _ply_move(self):
        assert self.sims == self.select_steps
        self.log.append((self.idx, "move"))

    def _ply_finish(self, on_moves=None, refill=True, game_offset=0):
        self.log.append((self.idx, "finish"))
        return super()._ply_finish(on_moves if on_moves is not None else (lambda m: None), refill, game_offset)


def _staggered_engine(log, rates=(1, 1)):
    from self_play_reinforcement_learning_amd.engine import LanedEngine

    eng = LanedEngine.__new__(LanedEngine)  # lanes without a GPU: no streams, fake arenas
    eng.lanes = [_SeqLane(log, i, rate=r) for i, r in enumerate(rates)]
    eng.streams = [None] * len(rates)
    eng.select_steps = 4
    eng.device = torch.device("cpu")
    eng.stagger = True
    eng._pending = False
    return eng


def test_staggered_lanes_keep_each_lanes_ply_order():
    """LanedEngine(stagger=True): lane 1 runs S / 2 simulation steps behind lane 0, so its ply ends (move,
    finish: the host round trip) and its next ply begins in the middle of lane 0's ply; each lane still runs
    begin -> steps 0..S-1 -> move -> finish per ply, every call after the first finishes one ply of each
    lane, and drain() completes lane 1's ply in flight."""
    log = []
    eng = _staggered_engine(log)
    for _ in range(3):
        eng.ply()
    assert eng._pending
    per = {i: [x for j, x in log if j == i] for i in (0, 1)}
    ply = ["begin", 0, 1, 2, 3, "move", "finish"]
    assert per[0] == ply * 3
    assert per[1] == ply * 2 + ["begin", 0, 1]  # lane 1's third ply is in flight
    # the issue order of a call (S = 4, lag 2): lane 0's ply up to its move with lane 1's last 2 steps,
    # then lane 1's move, finish, next begin and its first 2 steps, then lane 0's finish
    call2 = log[log.index((0, "finish")) + 1:]
    assert call2[:11] == [(0, "begin"), (0, 0), (1, 2), (0, 1), (1, 3), (0, 2), (0, 3), (0, "move"),
                          (1, "move"), (1, "finish"), (1, "begin")]
    assert call2[11:14] == [(1, 0), (1, 1), (0, "finish")]
    eng.drain()
    assert not eng._pending
    per1 = [x for j, x in log if j == 1]
    assert per1 == ply * 3 and [ln.plies_run for ln in eng.lanes] == [3, 3]


def test_staggered_play_games_single_process():
    """play_games with staggered lanes: a ply in flight is completed before the games are set up and after
    the last ply, every game's records reach the sink once, and both lanes end at a ply boundary."""
    log = []
    eng = _staggered_engine(log, rates=(2, 1))
    eng.ply()  # a ply() run leaves lane 1 part-way through its ply ...
    assert eng._pending
    got = []
    eng.play_games(6, on_moves=lambda m: got.extend(m["game"].tolist()))  # ... play_games completes it first
    assert not eng._pending
    assert [ln.games_done for ln in eng.lanes] == [3, 3]
    S = eng.GAME_ID_STRIDE
    assert sorted(got) == sorted([0, 1, 2] + [S + i for i in range(3)])
    per1 = [x for j, x in log if j == 1]
    assert per1 == ["begin", 0, 1, 2, 3, "move", "finish"] * eng.lanes[1].plies_run


def test_staggered_refresh_network_finishes_the_ply_in_flight():
    """LanedEngine.refresh_network with a staggered ply in flight: without a Move sink it refuses (the
    drained ply's finished games would be dropped); with one it completes the ply on the old weights first,
    then refreshes every lane -- no search mixes two weight versions."""
    log = []
    eng = _staggered_engine(log)
    for ln in eng.lanes:
        ln.refresh_network = (lambda ln=ln: log.append((ln.idx, "refresh")))
    eng.ply()
    assert eng._pending
    with pytest.raises(RuntimeError):
        eng.refresh_network()
    eng.refresh_network(on_moves=lambda m: None)
    assert not eng._pending
    assert log[-2:] == [(0, "refresh"), (1, "refresh")]
    assert log.index((1, "finish"), log.index((0, "finish")) + 1) < log.index((0, "refresh"))


def test_pack_unpack_roundtrip():
    m = _moves(0, 9)
    back = D.unpack_moves(D.pack_moves(m), 42, 7)
    for k in m:
        assert torch.equal(back[k].reshape(m[k].shape), m[k]), k


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_primitives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_restore(q.get(timeout=120)) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [sum(r + 1 for r in range(world)), sum(10 * r for r in range(world)), world, 0, 0, 0, world, 0]
    assert all(r[1] == want for r in res)
    assert all(r[3] == 1.5 * (world - 1) for r in res)
    assert all(r[4] == 0.0 for r in res)  # rank 0's weights everywhere
    assert all(r[5] == [1.0, 7] for r in res)  # float buffers and the int64 counter too


def test_end_ply_single_process():
    """Without a process group every ply returns (done, stats): this process's statistics on round
    plies (every `every`-th, or forced), None on the others; the sink gets the rows at once."""
    got = []
    ex = D.MoveExchange(42, 7, sink=lambda m: got.append(int(m["z"].shape[0])), every=3)
    calls = []

    def stats():
        calls.append(1)
        return [5, 6]

    out = []
    for ply in range(4):
        ex.stage(_moves(ply, ply))
        out.append(ex.end_ply(stats, done=ply == 3))
    out.append(ex.end_ply(stats, done=True, force=True))
    assert out == [(False, None), (False, None), (False, [5, 6]), (True, None), (True, [5, 6])]
    assert len(calls) == 2
    assert got == [1, 2, 3] and ex.rows_gathered == 6


def test_rank_env_and_device_check(monkeypatch):
    env = D.rank_env(3, 8, 12345, base={"X": "1"})
    assert env == {"X": "1", "RANK": "3", "LOCAL_RANK": "3", "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8",
                   "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "12345"}
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.delenv("SPMCTS_ALLOW_OVERSUBSCRIBE", raising=False)
    with pytest.raises(RuntimeError, match="only 1 GPU"):
        D.check_devices(8)
    monkeypatch.setenv("SPMCTS_ALLOW_OVERSUBSCRIBE", "1")
    assert D.check_devices(8) == 1


_CHILD = """
import os, sys, torch.distributed as dist
sys.path.insert(0, {repo!r})
from self_play_reinforcement_learning_amd import distributed as D
rank, world, local = D.init_from_env(backend="gloo")
s = D.all_reduce_stats([1, rank])
open(os.path.join({out!r}, "rank%d" % rank), "w").write(" ".join(
    [os.environ["RANK"], os.environ["LOCAL_RANK"], os.environ["WORLD_SIZE"], os.environ["MASTER_ADDR"],
     str(world), str(D.is_distributed())] + [str(int(x)) for x in s]))
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == rank and 3 or 0)
"""


def test_launch_script_wires_ranks(tmp_path):
    """bench.py's self-launch: N child processes of one script with torchrun's environment, one
    rendezvous on 127.0.0.1, a collective across them; a failing rank's exit code comes back."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "child.py"
    script.write_text(_CHILD.format(repo=repo, out=str(tmp_path)))
    assert D.launch_script([str(script)], 3) == 0
    for r in range(3):
        f = (tmp_path / f"rank{r}").read_text().split()
        assert f == [str(r), str(r), "3", "127.0.0.1", "3", "True", "3", "3"]
    os.environ["FAIL_RANK"] = "1"
    try:
        assert D.launch_script([str(script)], 2) == 3
    finally:
        del os.environ["FAIL_RANK"]


def _spawn_target(out, tag):
    rank, world, _ = D.init_from_env(backend="gloo")
    s = D.all_reduce_stats([rank])
    with open(os.path.join(out, f"{tag}{rank}"), "w") as f:
        f.write(f"{rank} {world} {int(s[0])}")
    torch.distributed.destroy_process_group()
    if tag == "fail" and rank == 1:
        raise SystemExit(5)


def test_spawn_ranks(tmp_path):
    """SelfPlayScheduler's self-spawn: fn runs in N spawned processes as ranks 0..N-1."""
    D.spawn_ranks(_spawn_target, 2, str(tmp_path), "ok")
    assert sorted((tmp_path / f"ok{r}").read_text() for r in range(2)) == ["0 2 1", "1 2 1"]
    with pytest.raises(RuntimeError, match="failed"):
        D.spawn_ranks(_spawn_target, 2, str(tmp_path), "fail")


def _spawn_slow_or_fail(out):
    """Rank 1 fails at once; rank 0 would wait for a minute (as in a collective whose peer is gone)."""
    import time

    rank = int(os.environ["RANK"])
    if rank == 1:
        raise SystemExit(7)
    time.sleep(60)


def test_spawn_ranks_fails_fast(tmp_path):
    """A rank that dies while rank 0 is still busy ends the whole call at once (the survivors are
    terminated), not after rank 0 finishes or the backend's collective timeout."""
    import time

    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match=r"\(1, 7\)"):
        D.spawn_ranks(_spawn_slow_or_fail, 2, str(tmp_path))
    assert time.monotonic() - t0 < 45


def _report_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      SPMCTS_DIST_INIT="file://" + port)
    D.init_from_env(backend="gloo")
    ex = D.MoveExchange(42, 7, every=2)
    for ply in range(4):
        ex.stage(_moves(rank + ply, rank + 1))
        ex.end_ply(lambda: [ply], done=False)
    rep = D.rank_report([100.0 * (rank + 1), 2.0, ex.rounds, ex.seconds / max(1, ex.rounds) * 1e3, ex.rows_gathered])
    q.put((rank, rep))
    torch.distributed.destroy_process_group()


def test_rank_report_gloo():
    """bench.py's per-rank lines: every rank gets every rank's row (positions/s, timed seconds,
    exchange rounds, ms per round, rows received), in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    rows = res[0]
    assert [r[0] for r in rows] == [100.0, 200.0] and all(r[1] == 2.0 for r in rows)
    assert all(r[2] == 2 and r[3] >= 0 for r in rows)  # two exchange rounds (every 2 of 4 plies)
    assert rows[0][4] == 4 * 1 + 4 * 2 and rows[1][4] == 0  # rows reach rank 0 only
    assert D.rank_report([1.0, 2.0]) == [[1.0, 2.0]]  # no process group: this process's row


def test_overlap_needs_weight_snapshot():
    """The trainer's own stream is used only when every self-play evaluator reads a snapshot of the
    weights; an evaluator on the live module keeps the SGD steps on the plies' stream (no race)."""
    import types

    from self_play_reinforcement_learning_amd import evaluator as E
    from self_play_reinforcement_learning_amd.engine import SelfPlayEngine
    from self_play_reinforcement_learning_amd.self_play_parallel import SelfPlayScheduler

    assert E.HipTowerEvaluator.snapshot and E.TableEvaluator.snapshot
    assert not E.ModuleEvaluator.snapshot and not E.CallableEvaluator.snapshot
    fake = types.SimpleNamespace(evaluator=E.ModuleEvaluator(torch.nn.Identity()), evaluator1=None)
    assert SelfPlayEngine.weights_snapshot.fget(fake) is False
    fake.evaluator = E.TableEvaluator(None)
    assert SelfPlayEngine.weights_snapshot.fget(fake) is True
    sp = SelfPlayScheduler.__new__(SelfPlayScheduler)
    sp.overlap_training = True
    sp.engine = types.SimpleNamespace(weights_snapshot=False)
    assert not sp._overlap_ok()
    sp.engine = types.SimpleNamespace(weights_snapshot=True)
    assert sp._overlap_ok()
    sp.overlap_training = False
    assert not sp._overlap_ok()


def _exchange_worker(rank, world, port, q):
    # SPMCTS_DIST_SINGLE: world size 1 runs the same collectives (the 1-GPU RCCL rehearsal's mode)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      SPMCTS_DIST_INIT="file://" + port, SPMCTS_DIST_SINGLE="1")
    D.init_from_env(backend="gloo")
    assert D.is_distributed()
    got = []
    ex = D.MoveExchange(42, 7, sink=lambda m: got.append({k: v.clone() for k, v in m.items()}), every=3)
    out = []
    for ply in range(7):
        ex.stage(_moves(10 * rank + ply, (rank + ply) % 3))  # 0..2 records per ply, some plies none
        out.append(ex.end_ply(lambda: [rank, ply], done=ply >= 2 + rank))
    out.append(ex.end_ply(lambda: [rank, 99], done=True, force=True))
    q.put(_by_value((rank, out, got, ex.rounds)))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_move_exchange_rounds_gloo(world):
    """Rounds every 3 plies (+ one forced): None between rounds; at a round every rank sees the
    same (all-done, summed stats); rank 0 receives exactly the rows staged since the previous round,
    rank by rank, bit-exact after the device pack/unpack; the other ranks' sinks are never called.
    World size 1 runs under SPMCTS_DIST_SINGLE=1 (a process group and every collective of one rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([_restore(q.get(timeout=120)) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, out, got, rounds in res:
        assert rounds == 3
        assert [o is None for o in out] == [True, True, False, True, True, False, True, False]
    for i in (2, 5, 7):
        assert len({str(r[1][i]) for r in res}) == 1  # identical on every rank
    ply2, ply5, last = res[0][1][2], res[0][1][5], res[0][1][7]
    assert ply2 == (world == 1, [sum(range(world)), 2 * world])
    assert ply5[0] == (5 >= 2 + world - 1) and ply5[1] == [sum(range(world)), 5 * world]
    assert last == (True, [sum(range(world)), 99 * world])
    assert all(r[2] == [] for r in res[1:])
    got = res[0][2]
    batches = [(0, 3), (3, 6), (6, 7)]
    nonempty = []
    for lo, hi in batches:
        parts = [_moves(10 * r + p, (r + p) % 3) for r in range(world) for p in range(lo, hi)]
        parts = [m for m in parts if m["z"].shape[0]]
        if parts:
            nonempty.append({k: torch.cat([m[k] for m in parts]) for k in parts[0]})
    assert len(got) == len(nonempty)
    for g, e in zip(got, nonempty):
        for k in e:
            assert torch.equal(g[k].reshape(e[k].shape), e[k]), k


def test_scheduler_rank_count_and_spawn_kwargs(tmp_path, monkeypatch):
    """SelfPlayScheduler(gpus=...): how many rank processes train_model / compare_models start (1 inside
    a launched job; else the call's gpus, the constructor's, 1 (in-process) by default, every visible GPU
    for gpus="all"), and the constructor
    arguments the ranks rebuild it from (networks as host copies, one start_time, gpus=1) pickle."""
    import pickle

    from self_play_reinforcement_learning_amd import ModelContainer, ResidualTower
    from self_play_reinforcement_learning_amd.envs import Connect4Env
    from self_play_reinforcement_learning_amd.mcts import MCTreeSearch
    from self_play_reinforcement_learning_amd.self_play_parallel import SelfPlayScheduler

    for k in ("WORLD_SIZE", "RANK"):
        monkeypatch.delenv(k, raising=False)
    net = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=4)
    ev = ModelContainer(MCTreeSearch, policy_kwargs=dict(network=ResidualTower(7, 6, 7, num_blocks=1, filter_factor=4),
                                                          env=Connect4Env, iterations=10))
    sp = SelfPlayScheduler(ModelContainer(MCTreeSearch, policy_kwargs=dict(env=Connect4Env, iterations=10)),
                           Connect4Env, evaluation_policy_container=ev, network=net, save_dir=str(tmp_path), gpus=3)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert sp._ranks(None) == 3 and sp._ranks(2) == 2 and sp._ranks(1) == 1
    sp.gpus = None
    assert sp._ranks(None) == 1  # in this process unless asked
    assert sp._ranks("all") == 8
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "0")
    assert sp._ranks(4) == 1  # already one rank of a launched job
    kw = pickle.loads(pickle.dumps(sp._spawn_kwargs()))
    assert kw["gpus"] == 1 and kw["start_time"] == sp.start_time and kw["device"] is None
    assert kw["network"] is not net and torch.equal(kw["network"].conv1.weight, net.conv1.weight)
    assert kw["evaluation_policy_container"].policy_kwargs["iterations"] == 10
    assert isinstance(kw["evaluation_policy_container"].policy_kwargs["network"], ResidualTower)


def test_launch_script_refuses_a_gpu_initialised_parent(monkeypatch):
    """launch_script (bench.py --gpus N) starts the rank processes only from a parent that has not initialised
    HIP; with torch.cuda.is_initialized() True it raises before starting anything."""
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    with pytest.raises(RuntimeError, match="initialised the GPU"):
        D.launch_script(["-c", "raise SystemExit(3)"], 2)
    monkeypatch.undo()
    assert not torch.cuda.is_initialized()
    assert D.launch_script(["-c", "raise SystemExit(0)"], 2) == 0
