"""Host replay memory with the reference's `Memory` API (rl_utils/memory.py:8-94).

The batched self-play path does not use this class: the scheduler appends the
arena's exported Move rows to `replay.DeviceReplay`, a device ring.  `Memory` is
the host-side object that single-tree `MCTreeSearch` users (and code written
against the reference) hold; its observable behaviour is pinned by the G7
fixture (tests/golden/memory_ops.json, made by running the reference's Memory):

  * `Memory(max_size)` — a bounded ring (None = unbounded) evicting the oldest
    record, like the reference's deque(maxlen) (:9-12, :17-20);
  * `sample(k)` — `np.random.choice(arange(len), k, replace=False)` over the
    records oldest-first, so the global numpy stream picks the same records as
    the reference's (:26-30);
  * `change_size(n)` keeps the newest n (:22-24); `reset()` empties (:32-33);
  * `get_duplicates(key)` — groups of record indices per distinct key (:35-45);
  * `deduplicate(key, values, named_tuple, maxlen)` (:47-53, Deduplicator
    :56-94): records with equal `key` bytes collapse into one whose `values` are
    the running sums / counts, groups in first-seen order.  The group table
    persists across calls (records added after a deduplicate are folded in at
    the next call; evicted records stay counted), and the new records carry
    only `key` and `values`, so a named tuple with other required fields (the
    reference's own `Move`, mcts.py:17, via MCTreeSearch.deduplicate
    mcts.py:385-386) raises TypeError and leaves the buffer in place — as in
    the reference, including its aliasing: sums accumulate in place into the
    first record's tensors, so after that TypeError the first record of each
    duplicated key holds the group's sums.
"""
import logging
from collections import defaultdict

import numpy as np
import torch


class Memory:
    def __init__(self, max_size=None):
        self.max_size = max_size
        self._cap = max_size  # ring bound (deduplicate(maxlen=...) rebinds it, not max_size)
        self._ring = []      # physical slots
        self._start = 0      # slot of the oldest record once the ring is full
        self.deduplicator = None

    # ------------------------------------------------------------------ ring
    def _records(self):
        """Records oldest-first."""
        return self._ring[self._start:] + self._ring[:self._start]

    def _load(self, records):
        records = list(records)
        if self._cap is not None:
            records = records[len(records) - min(len(records), self._cap):]
        self._ring, self._start = records, 0

    @property
    def _buffer(self):
        return self._records()

    def __len__(self):
        return len(self._ring)

    def __iter__(self):
        return iter(self._records())

    def __getitem__(self, i):
        n = len(self._ring)
        if not -n <= i < n:
            raise IndexError("Memory index out of range")
        return self._ring[(self._start + (i % n)) % n]

    def add(self, experience):
        if self._cap is None or len(self._ring) < self._cap:
            self._ring.append(experience)
        elif self._cap > 0:
            self._ring[self._start] = experience
            self._start = (self._start + 1) % self._cap
        if self.deduplicator is not None:
            self.deduplicator.add_temp(experience)

    def add_batch(self, experiences):
        for e in experiences:
            self.add(e)

    def change_size(self, max_size):
        records = self._records()
        self.max_size = self._cap = max_size
        self._load(records)

    def sample(self, batch_size):
        pick = np.random.choice(np.arange(len(self._ring)), size=batch_size, replace=False)
        return [self[int(i)] for i in pick]

    def reset(self):
        self._cap = self.max_size
        self._ring, self._start = [], 0

    # ------------------------------------------------------------------ duplicates
    def get_duplicates(self, key):
        records = self._records()
        keys = torch.stack([getattr(r, key) for r in records], dim=0)
        unique_keys, inverse = torch.unique(keys, return_inverse=True, dim=0)
        groups = defaultdict(list)
        for idx, g in enumerate(inverse.tolist()):
            groups[g].append(idx)
        logging.info(f"{len(groups)} different entries for {len(records)} entries")
        return groups, unique_keys

    def deduplicate(self, key, values, named_tuple, maxlen=None):
        if self.deduplicator is None:
            self.deduplicator = Deduplicator(key, values, named_tuple, buffer=self._records())
        logging.info(f"len of old buffer is {len(self)}")
        merged = self.deduplicator.deduplicate(max_size=maxlen)
        self._cap = maxlen  # the rebuilt buffer is bounded by maxlen (None: unbounded), max_size kept
        self._load(merged)
        logging.info(f"len of new buffer is {len(self)}")


class _Group:
    __slots__ = ("count", "key", "sums")

    def __init__(self, key, vals):
        self.count, self.key, self.sums = 1, key, list(vals)

    def fold(self, vals):
        self.count += 1
        for i, v in enumerate(vals):
            self.sums[i] += v  # in place for tensors: the group's first record accumulates, as in the reference


class Deduplicator:
    """Persistent state-keyed group table behind Memory.deduplicate (rl_utils/memory.py:56-94)."""

    def __init__(self, key, values, named_tuple, buffer=None):
        self.key = key
        self.values = list(values)
        self.named_tuple = named_tuple
        self._groups = {}                         # key bytes -> _Group, first-seen order
        self._pending = list(buffer) if buffer else []

    def add_temp(self, experience):
        self._pending.append(experience)

    def add(self, experience):
        k = getattr(experience, self.key)
        tag = k.detach().cpu().numpy().tobytes()
        vals = [getattr(experience, v) for v in self.values]
        g = self._groups.get(tag)
        if g is None:
            self._groups[tag] = _Group(k, vals)
        else:
            g.fold(vals)

    def deduplicate(self, max_size=None):
        pending, self._pending = self._pending, []
        for e in pending:
            self.add(e)
        return self.create_memory(max_size=max_size)

    def create_memory(self, max_size=None):
        out = []
        for g in self._groups.values():
            fields = {self.key: g.key}
            fields.update({v: s / g.count for v, s in zip(self.values, g.sums)})
            out.append(self.named_tuple(**fields))
        if max_size is not None:
            out = out[len(out) - min(len(out), max_size):]
        return out
