"""Replay memory with the reference API (rl_utils/memory.py:8-94).

`Memory(max_size)`: deque(maxlen), `add`, `sample(k)` (uniform without
replacement via np.random.choice, :26-30), `change_size`, `reset`, `len`,
`deduplicate(key, values, named_tuple)` (averaging duplicate states).
`add_batch` is new: it appends the arena's exported Move rows in one call.
"""
import logging
from collections import defaultdict, deque

import numpy as np
import torch


class Memory:
    def __init__(self, max_size=None):
        self.max_size = max_size
        self._buffer = deque(maxlen=max_size)
        self.deduplicator = None

    def __len__(self):
        return len(self._buffer)

    def add(self, experience):
        self._buffer.append(experience)
        if self.deduplicator:
            self.deduplicator.add_temp(experience)

    def add_batch(self, experiences):
        for e in experiences:
            self.add(e)

    def change_size(self, max_size):
        self.max_size = max_size
        self._buffer = deque(self._buffer, maxlen=max_size)

    def sample(self, batch_size):
        index = np.random.choice(np.arange(len(self._buffer)), size=batch_size, replace=False)
        return [self._buffer[i] for i in index]

    def reset(self):
        self._buffer = deque(maxlen=self.max_size)

    def get_duplicates(self, key):
        groups = defaultdict(list)
        keys = torch.stack([getattr(item, key) for item in self._buffer], dim=0)
        unique_keys, inverse = torch.unique(keys, return_inverse=True, dim=0)
        for i, item in enumerate(inverse):
            groups[int(item)].append(i)
        return groups, unique_keys

    def deduplicate(self, key, values, named_tuple, maxlen=None):
        if not self.deduplicator:
            self.deduplicator = Deduplicator(key=key, values=values, named_tuple=named_tuple, buffer=self._buffer)
        logging.info(f"len of old buffer is {len(self._buffer)}")
        self._buffer = self.deduplicator.deduplicate(max_size=maxlen)
        logging.info(f"len of new buffer is {len(self._buffer)}")


class Deduplicator:
    """Average `values` over experiences sharing the same `key` bytes (memory.py:56-94)."""

    def __init__(self, key, values, named_tuple, buffer=None):
        self.key = key
        self.values = values
        self.named_tuple = named_tuple
        self.counter = defaultdict(dict)
        self.temp_queue = deque(buffer) if buffer else deque()

    def deduplicate(self, max_size=None):
        for experience in self.temp_queue:
            self.add(experience)
        self.temp_queue = deque()
        return self.create_memory(max_size=max_size)

    def add_temp(self, experience):
        self.temp_queue.append(experience)

    def add(self, experience):
        k = getattr(experience, self.key).detach().cpu().numpy().tobytes()
        count = self.counter[k]
        if count:
            count["count"] += 1
            for v in self.values:
                count[v] = count[v] + getattr(experience, v)
        else:
            count["count"] = 1
            count[self.key] = getattr(experience, self.key)
            for v in self.values:
                count[v] = getattr(experience, v)

    def create_memory(self, max_size=None):
        buffer = deque(maxlen=max_size)
        for count in self.counter.values():
            kw = {self.key: count[self.key]}
            for v in self.values:
                kw[v] = count[v] / count["count"]
            for f in self.named_tuple._fields:
                kw.setdefault(f, None)
            buffer.append(self.named_tuple(**kw))
        return buffer
