"""CPU: the device replay ring (self_play_reinforcement_learning_amd/replay.py) against the
reference Memory semantics (rl_utils/memory.py): deque(maxlen) eviction, uniform sampling without
replacement, change_size keeping the newest rows.  Deduplication is pinned against the reference's own
outputs in test_memory_golden.py."""
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
