"""Device-resident replay ring: the trainer's side of the hot path without per-record host objects.

The reference moves every `Move` record through a multiprocessing queue into a
Python `deque` (rl_utils/memory.py:8-33) and samples `batch_size` of them per
update with `np.random.choice(len, k, replace=False)` (:26-30), stacking the
tensors again for the loss (mcts.py:234-252).  Here the arena's exported Move
rows (`Arena.export_moves` / `distributed.MoveExchange`: state int8 [n, cells],
tree_probs f32 [n, A], q f64 + dtype flag, z f32) are appended to fixed device
tensors, and a training batch is one uniform sample without replacement
(`torch.randperm`) gathered on the device.

The `Memory` surface is kept (`add`, `sample -> list[Move]`, `change_size`,
`reset`, `len`, `max_size`, `deduplicate`) so code written against the
reference's replay memory still works; the batched path is `add_moves` /
`sample_batch`.
"""
import torch

from .mcts import Move


class DeviceReplay:
    def __init__(self, max_size, width, height, n_actions, device=None):
        self.max_size = int(max_size)
        self.width, self.height, self.n_actions = width, height, n_actions
        self.cells = width * height
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._alloc(self.max_size)

    def _alloc(self, n):
        d = self.device
        self.state = torch.zeros((n, self.cells), dtype=torch.int8, device=d)
        self.probs = torch.zeros((n, self.n_actions), dtype=torch.float32, device=d)
        self.q = torch.zeros(n, dtype=torch.float64, device=d)
        self.q_f64 = torch.zeros(n, dtype=torch.uint8, device=d)
        self.z = torch.zeros(n, dtype=torch.float32, device=d)
        self.head = 0   # next write position
        self.count = 0

    def __len__(self):
        return self.count

    # ------------------------------------------------------------------ writes
    def add_moves(self, moves):
        """Append exported Move rows (dict of tensors, any device); oldest rows are evicted
        like deque(maxlen) (memory.py:11, :19-23)."""
        n = int(moves["z"].shape[0])
        if n == 0 or self.max_size == 0:
            return
        cols = dict(state=moves["state"].reshape(n, self.cells).to(self.device, torch.int8),
                    probs=moves["tree_probs"].reshape(n, self.n_actions).to(self.device, torch.float32),
                    q=moves["q"].reshape(n).to(self.device, torch.float64),
                    q_f64=moves.get("q_f64", torch.zeros(n, dtype=torch.uint8)).reshape(n).to(self.device,
                                                                                             torch.uint8),
                    z=moves["z"].reshape(n).to(self.device, torch.float32))
        if n > self.max_size:  # only the newest max_size survive
            cols = {k: v[n - self.max_size:] for k, v in cols.items()}
            n = self.max_size
        idx = (self.head + torch.arange(n, device=self.device)) % self.max_size
        for k, v in cols.items():
            getattr(self, k)[idx] = v
        self.head = (self.head + n) % self.max_size
        self.count = min(self.max_size, self.count + n)

    def add(self, move):
        """Memory.add(Move) (memory.py:19-23)."""
        q = torch.as_tensor(move.q)
        self.add_moves(dict(state=torch.as_tensor(move.state).reshape(1, -1),
                            tree_probs=torch.as_tensor(move.tree_probs).reshape(1, -1),
                            q=q.reshape(1).double(), q_f64=torch.tensor([1 if q.dtype == torch.float64 else 0]),
                            z=torch.as_tensor(move.actual_val).reshape(1).float()))

    # ------------------------------------------------------------------ reads
    def _order(self):
        """Physical indices of the live rows, oldest first."""
        start = (self.head - self.count) % self.max_size
        return (start + torch.arange(self.count, device=self.device)) % self.max_size

    def sample_batch(self, batch_size, generator=None):
        """Uniform sample without replacement (memory.py:26-30) -> (state int64 [k, W, H],
        z f32 [k], tree_probs f32 [k, A], q f32 [k]) on the device."""
        if batch_size > self.count:
            raise ValueError(f"cannot sample {batch_size} rows from {self.count}")
        pick = torch.randperm(self.count, device=self.device, generator=generator)[:batch_size]
        idx = self._order()[pick]
        s = self.state[idx].to(torch.int64).view(batch_size, self.width, self.height)
        return s, self.z[idx], self.probs[idx], self.q[idx].float()

    def sample(self, batch_size):
        """Memory.sample -> list of Move (dtypes as the reference's records, mcts.py:282-288, :230)."""
        pick = torch.randperm(self.count)[:batch_size].to(self.device)
        idx = self._order()[pick].cpu()
        st, pr = self.state.cpu(), self.probs.cpu()
        q, qf, z = self.q.cpu(), self.q_f64.cpu(), self.z.cpu()
        out = []
        for i in idx.tolist():
            qt = torch.tensor(float(q[i]), dtype=torch.float64 if qf[i] else torch.float32)
            out.append(Move(st[i].to(torch.int64).view(self.width, self.height), z[i].clone(), pr[i].clone(), qt))
        return out

    # ------------------------------------------------------------------ maintenance
    def change_size(self, max_size):
        """Memory.change_size (memory.py:22-24): keep the newest rows."""
        keep = self._order()[-min(self.count, int(max_size)):] if self.count else None
        rows = None if keep is None else dict(state=self.state[keep], tree_probs=self.probs[keep], q=self.q[keep],
                                              q_f64=self.q_f64[keep], z=self.z[keep])
        self.max_size = int(max_size)
        self._alloc(self.max_size)
        if rows is not None:
            self.add_moves(rows)

    def reset(self):
        self._alloc(self.max_size)

    # ------------------------------------------------------------------ snapshot / resume
    # The UpdateWorker pickles its whole Memory object (updateworker.py:127-139) and unpickles it on
    # resume (base_worker.py:36-41).  The ring is saved instead as plain tensors -- the physical
    # arrays, the write head, the live count and the shape -- so a snapshot loads with
    # torch.load(weights_only=True) (nothing in the file is executed) and restores the ring row for
    # row, eviction order included.
    FIELDS = ("state", "probs", "q", "q_f64", "z")

    def snapshot(self):
        """The ring as a dict of host tensors (torch.save-able)."""
        sd = {k: getattr(self, k).detach().cpu().clone() for k in self.FIELDS}
        sd["meta"] = torch.tensor([self.max_size, self.head, self.count, self.width, self.height, self.n_actions],
                                  dtype=torch.int64)
        return sd

    def load_snapshot(self, sd):
        """Restore a `snapshot()` (its capacity replaces this ring's, as the reference's unpickled
        Memory replaces the policy's)."""
        max_size, head, count, w, h, a = (int(x) for x in sd["meta"].tolist())
        if (w, h, a) != (self.width, self.height, self.n_actions):
            raise ValueError(f"replay snapshot is for a {w}x{h} board with {a} actions, "
                             f"not {self.width}x{self.height} with {self.n_actions}")
        if not (0 <= count <= max_size and 0 <= head < max(1, max_size)):
            raise ValueError(f"corrupt replay snapshot: max_size {max_size}, head {head}, count {count}")
        shapes = dict(state=(max_size, self.cells), probs=(max_size, a), q=(max_size,), q_f64=(max_size,),
                      z=(max_size,))
        for k in self.FIELDS:
            if tuple(sd[k].shape) != shapes[k]:
                raise ValueError(f"replay snapshot field {k}: shape {tuple(sd[k].shape)}, expected {shapes[k]}")
        self.max_size = max_size
        self._alloc(max_size)
        for k in self.FIELDS:
            getattr(self, k).copy_(sd[k])
        self.head, self.count = head, count

    def save(self, path):
        torch.save(self.snapshot(), path)

    def load(self, path):
        self.load_snapshot(torch.load(path, weights_only=True, map_location="cpu"))

    def deduplicate(self, key="state", values=("actual_val", "tree_probs"), named_tuple=None, maxlen=None):
        """Memory.deduplicate (memory.py:35-94, Deduplicator): rows with identical boards merge into
        one whose z and tree_probs (and q) are the group means; groups keep first-occurrence order.
        Runs on the device: torch.unique over the int8 board rows + index_add."""
        if key != "state":
            raise ValueError("only state-keyed deduplication is supported")
        if self.count == 0:
            return
        order = self._order()
        st = self.state[order]
        uniq, inv = torch.unique(st, dim=0, return_inverse=True)
        g = uniq.shape[0]
        n = torch.zeros(g, dtype=torch.float64, device=self.device).index_add_(
            0, inv, torch.ones(self.count, dtype=torch.float64, device=self.device))
        zs = torch.zeros(g, dtype=torch.float64, device=self.device).index_add_(0, inv, self.z[order].double())
        ps = torch.zeros((g, self.n_actions), dtype=torch.float64, device=self.device).index_add_(
            0, inv, self.probs[order].double())
        qs = torch.zeros(g, dtype=torch.float64, device=self.device).index_add_(0, inv, self.q[order])
        first = torch.full((g,), self.count, dtype=torch.int64, device=self.device).scatter_reduce_(
            0, inv, torch.arange(self.count, device=self.device), reduce="amin")
        rank = torch.argsort(first)
        rows = dict(state=uniq[rank], tree_probs=(ps / n[:, None])[rank].float(), q=(qs / n)[rank],
                    q_f64=torch.zeros(g, dtype=torch.uint8, device=self.device), z=(zs / n)[rank].float())
        size = self.max_size if maxlen is None else int(maxlen)
        self.max_size = size
        self._alloc(size)
        self.add_moves(rows)
