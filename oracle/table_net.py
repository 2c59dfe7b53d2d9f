"""Deterministic "table network" used to make MCTS bit-exactly checkable.

TEST INFRASTRUCTURE (see oracle/__init__.py).  The reference's leaf evaluator
protocol is `net(state int64[W,H], player) -> (list[A] probs, float v)`
(games/general/modules.py:109-112, games/algos/inference_proxy.py:21-24):
the board is multiplied by `player` (so +1 = own pieces), evaluated, and the
value is multiplied back by `player`.  A real ResNet cannot be reproduced bit
for bit across CPU/GPU, so parity of the *search* is pinned with this net,
whose outputs are an exactly-computable function of the encoded board:

  cells c_i in [x][y] order, c = 0 empty / 1 own / 2 enemy
  h      = FNV-1a-style fold over (c_i + 3 i + 1) ^ salt
  k_j    = 1 + ((splitmix64(h + j) >> 40) & 0xFFFF)          (j < A)
  prob_j = float32(k_j) / float32(sum_j k_j)                 (IEEE fp32 div)
  value  = float32(((splitmix64(h ^ 0x5DEECE66D) >> 40) & 0xFFFF) - 32768) / 32768

The identical function is implemented as a HIP kernel in the product library
(`spmcts_table_net`) so that GPU searches can be compared bit for bit.
"""
import numpy as np

MASK64 = (1 << 64) - 1
FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def cells_of(board_times_player):
    """Encode a board already multiplied by the mover: 0 empty, 1 own(+1), 2 enemy(-1)."""
    b = np.asarray(board_times_player).reshape(-1)
    out = np.zeros(b.shape, dtype=np.int64)
    out[b == 1] = 1
    out[b == -1] = 2
    return out


def table_eval(cells, n_actions, salt=0):
    h = FNV_OFFSET
    for i, c in enumerate(cells):
        h = ((h ^ (int(c) + 3 * i + 1)) * FNV_PRIME) & MASK64
    h ^= salt & MASK64
    ks = [1 + ((splitmix64((h + j) & MASK64) >> 40) & 0xFFFF) for j in range(n_actions)]
    total = np.float32(sum(ks))
    probs = np.array(ks, dtype=np.float32) / total
    raw = ((splitmix64(h ^ 0x5DEECE66D) >> 40) & 0xFFFF) - 32768
    value = np.float32(raw) / np.float32(32768.0)
    return probs.astype(np.float32), np.float32(value)


class TableNet:
    """Callable with the reference network protocol (modules.py:109-112)."""

    def __init__(self, n_actions, salt=0):
        self.n_actions = n_actions
        self.salt = salt
        self.calls = 0

    def __call__(self, state, player=1):
        self.calls += 1
        s = np.asarray(state) * player
        probs, v = table_eval(cells_of(s), self.n_actions, self.salt)
        return [float(p) for p in probs], float(v) * player

    # no-op torch.nn.Module-ish surface used by MCTreeSearch.__init__ (mcts.py:138,390)
    def to(self, *a, **k):
        return self

    def train(self, *a, **k):
        return self

    def share_memory(self):
        return self
