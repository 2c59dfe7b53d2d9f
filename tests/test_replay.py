"""CPU: the device replay ring (self_play_reinforcement_learning_amd/replay.py) against the
reference Memory semantics (rl_utils/memory.py): deque(maxlen) eviction, uniform sampling without
replacement, change_size keeping the newest rows.  Deduplication is pinned against the reference's own
outputs in test_memory_golden.py."""
import os
from collections import deque

import numpy as np
import torch

from self_play_reinforcement_learning_amd.mcts import Move
from self_play_reinforcement_learning_amd.replay import DeviceReplay


def _moves(n, seed=0, dup_every=0):
    g = torch.Generator().manual_seed(seed)
    st = torch.randint(-1, 2, (n, 42), dtype=torch.int8, generator=g)
    if dup_every:
        st[dup_every::dup_every] = st[0]
    return dict(state=st, tree_probs=torch.rand(n, 7, generator=g), q=torch.rand(n, generator=g, dtype=torch.float64),
                q_f64=torch.zeros(n, dtype=torch.uint8), z=torch.randint(-1, 2, (n,), generator=g).float())


def test_ring_eviction_matches_deque():
    r = DeviceReplay(50, 7, 6, 7)
    ref = deque(maxlen=50)
    for chunk, seed in ((30, 1), (15, 2), (40, 3), (0, 4), (70, 5)):
        m = _moves(chunk, seed)
        r.add_moves(m)
        for i in range(chunk):
            ref.append(float(m["z"][i]) + 10 * float(m["tree_probs"][i, 0]))
        live = r._order()
        got = (r.z[live] + 10 * r.probs[live, 0]).tolist()
        assert len(r) == len(ref)
        np.testing.assert_allclose(got, list(ref), rtol=0, atol=1e-6)


def test_sample_batch_is_uniform_without_replacement():
    r = DeviceReplay(100, 7, 6, 7)
    m = _moves(100, 7)
    m["z"] = torch.arange(100).float()
    r.add_moves(m)
    counts = np.zeros(100)
    for _ in range(400):
        s, z, p, q = r.sample_batch(25)
        assert s.shape == (25, 7, 6) and s.dtype == torch.int64 and p.shape == (25, 7) and q.dtype == torch.float32
        zz = z.long().numpy()
        assert len(set(zz.tolist())) == 25  # no replacement
        counts[zz] += 1
    assert abs(counts.mean() - 100) < 1e-9 and counts.min() > 60 and counts.max() < 140


def test_sample_returns_reference_moves():
    r = DeviceReplay(10, 7, 6, 7)
    r.add_moves(_moves(10, 3))
    ms = r.sample(4)
    assert len(ms) == 4 and all(isinstance(m, Move) for m in ms)
    assert ms[0].state.shape == (7, 6) and ms[0].state.dtype == torch.int64
    assert ms[0].tree_probs.shape == (7,) and ms[0].actual_val.dtype == torch.float32 and ms[0].q.dtype == torch.float32


def test_change_size_keeps_newest():
    r = DeviceReplay(20, 7, 6, 7)
    m = _moves(20, 4)
    r.add_moves(m)
    r.change_size(8)
    assert len(r) == 8
    np.testing.assert_array_equal(r.z[r._order()].numpy(), m["z"][-8:].numpy())
    r.change_size(30)
    assert len(r) == 8 and r.max_size == 30


def _ring_rows(r):
    live = r._order()
    return {k: getattr(r, k)[live].clone() for k in DeviceReplay.FIELDS}


def test_snapshot_roundtrip_restores_ring_row_for_row(tmp_path):
    """The replay snapshot (the UpdateWorker's save_memory / load_memory, updateworker.py:127-139,
    base_worker.py:36-41) holds tensors only (torch.load(weights_only=True)) and restores the ring
    exactly: physical arrays, head, count, capacity -- so the eviction order continues unchanged."""
    r = DeviceReplay(50, 7, 6, 7)
    for n, seed in ((30, 1), (45, 2), (7, 3)):  # wrapped: head mid-ring
        r.add_moves(_moves(n, seed))
    p = tmp_path / "memory-x:50"
    r.save(p)
    sd = torch.load(p, weights_only=True)
    assert set(sd) == set(DeviceReplay.FIELDS) | {"meta"}
    s = DeviceReplay(10, 7, 6, 7)
    s.load(p)
    assert (s.max_size, s.head, s.count) == (r.max_size, r.head, r.count) == (50, r.head, 50)
    for k in DeviceReplay.FIELDS:
        assert torch.equal(getattr(s, k), getattr(r, k)), k
    # both continue identically
    r.add_moves(_moves(9, 4))
    s.add_moves(_moves(9, 4))
    a, b = _ring_rows(r), _ring_rows(s)
    assert all(torch.equal(a[k], b[k]) for k in a)
    bad = DeviceReplay(5, 3, 3, 9)
    import pytest

    with pytest.raises(ValueError):
        bad.load(p)


def test_trainer_snapshots_every_50000_and_at_epoch_end(tmp_path):
    """UpdateWorker.pull's cadence (updateworker.py:119-125): a snapshot when the ring's length crosses a
    multiple of 50,000, the previous file removed (:136-139); none while the length stays put."""
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

    net = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=2)
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    t = _Trainer(net, opt, memory_size=120000, batch_size=8, min_memory=8, q_average=True, device="cpu")
    t.rows_added()
    assert not list(tmp_path.iterdir())  # no run_dir yet: nothing saved
    t.run_dir = str(tmp_path)

    def files():
        return sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("memory"))

    t.memory.add_moves(_moves(30000, 1))
    t.rows_added()
    assert files() == []
    t.memory.add_moves(_moves(30000, 2))  # 60,000: crosses 50,000
    t.rows_added()
    assert len(files()) == 1 and files()[0].endswith(":60000")
    t.memory.add_moves(_moves(30000, 3))  # 90,000: same band
    t.rows_added()
    assert len(files()) == 1 and files()[0].endswith(":60000")
    t.memory.add_moves(_moves(40000, 4))  # 120,000 (full): crosses 100,000
    t.rows_added()
    assert len(files()) == 1 and files()[0].endswith(":120000")
    t.memory.add_moves(_moves(40000, 5))  # full ring: length stays 120,000 -> no snapshot
    t.rows_added()
    assert files()[0].endswith(":120000")
    first = files()[0]
    saved = t.save_memory()  # the epoch-end snapshot: a new file, the previous one removed
    assert saved.endswith(":120000") and files() == [os.path.basename(saved)]
    assert os.path.basename(saved) == first or not (tmp_path / first).exists()
    assert not (tmp_path / ".memory.partial").exists()


def test_scheduler_resume_memory(tmp_path):
    """train_model(resume_memory=True) (self_play_parallel.py:213, updateworker.py:67-69): the newest
    snapshot of the newest earlier run replaces the trainer's ring, row for row; with no snapshot the
    ring stays empty (the reference logs its error and carries on)."""
    from self_play_reinforcement_learning_amd.envs import Connect4Env
    from self_play_reinforcement_learning_amd.mcts import MCTreeSearch
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.base_model import ModelContainer
    from self_play_reinforcement_learning_amd.self_play_parallel import SelfPlayScheduler

    def sched(start):
        net = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=2)
        c = ModelContainer(MCTreeSearch, policy_kwargs=dict(env=Connect4Env, iterations=10, memory_size=5000,
                                                            min_memory=10))
        return SelfPlayScheduler(c, Connect4Env, network=net, save_dir=str(tmp_path), start_time=start, device="cpu",
                                 evaluation_games=0)

    a = sched("2026-01-01T00:00:00")
    a.setup_update_worker(resume_memory=True)  # nothing to resume yet
    assert len(a.trainer.memory) == 0
    for n, seed in ((3000, 1), (3500, 2)):
        a.trainer.memory.add_moves(_moves(n, seed))
    a.trainer.rows_added()
    older = a.trainer.save_memory()
    a.trainer.memory.add_moves(_moves(100, 3))
    a.trainer.memory_size = len(a.trainer.memory)
    newest = a.trainer.save_memory()
    assert not os.path.exists(older) and os.path.exists(newest)
    b = sched("2026-01-02T00:00:00")
    b.setup_update_worker(resume_memory=True)
    ra, rb = a.trainer.memory, b.trainer.memory
    assert (rb.max_size, rb.head, rb.count) == (ra.max_size, ra.head, ra.count) == (5000, ra.head, 5000)
    for k in DeviceReplay.FIELDS:
        assert torch.equal(getattr(rb, k), getattr(ra, k)), k
    assert b.trainer.memory_size == 5000
    # training starts at once from the resumed ring (min_memory met)
    assert b.trainer.step() is not None


def test_scheduler_resume_memory_without_save_dir():
    """resume_memory / resume_model with save_dir=None: a warning and an empty ring (as with no snapshot),
    not a TypeError from the glob."""
    from self_play_reinforcement_learning_amd.envs import Connect4Env
    from self_play_reinforcement_learning_amd.mcts import MCTreeSearch
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.base_model import ModelContainer
    from self_play_reinforcement_learning_amd.self_play_parallel import SelfPlayScheduler

    net = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=2)
    c = ModelContainer(MCTreeSearch, policy_kwargs=dict(env=Connect4Env, iterations=10, memory_size=500,
                                                        min_memory=10))
    s = SelfPlayScheduler(c, Connect4Env, network=net, save_dir=None, device="cpu", evaluation_games=0)
    s.setup_update_worker(resume_memory=True, resume_model=True)
    assert len(s.trainer.memory) == 0
