"""Multi-GPU self-play: one process per GPU, games sharded, RCCL only at episode-batch ends.

The reference's only parallelism is CPU processes exchanging every leaf over
multiprocessing queues (games/algos/self_play_parallel.py:95-171,
rl_utils/queues.py).  Games are independent units (they share only frozen
weights within an epoch), so here every rank owns its own arena of game slots
and its own Philox subsequences (subsequence0 = rank * n_trees) and the data
path has no collective.  The exchange steps are the ones the reference has:

  * finished games' Move records go to the replay owner on rank 0
    (memory_queue -> UpdateWorker -> Memory, mcts.py:225-232,
    updateworker.py:119-125) and episode statistics (games finished,
    wins/draws/losses by side, self_play_parallel.py:302-327) are summed over
    ranks — both in ONE exchange round per episode batch (`MoveExchange`: every
    `every` plies and at the end of a run).  Between rounds each rank stages
    its finished games' packed Move rows on its own device; a round is one
    all_gather of a small int64 header per rank (row count, not-done flag,
    stats) and one `gather` of the padded rows to rank 0, where they are
    unpacked on the device and handed to the sink (the device replay ring);
  * weights are broadcast from rank 0 at epoch boundaries (the reference's
    checkpoint reload, selfplayworker.py:109-114).

backend "nccl" is RCCL on ROCm (xGMI between the GPUs of a node); the same
code runs on "gloo" for CPU tests.
"""
import os
import time

import torch
import torch.distributed as dist

STAT_FIELDS = ("games", "moves", "first_w", "first_d", "first_l", "second_w", "second_d", "second_l")


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def single_rank_group():
    """SPMCTS_DIST_SINGLE=1: a process group even at world size 1, with every collective of the
    multi-GPU path issued (rehearsal of the RCCL path on a 1-GPU box, where RCCL refuses two ranks
    on one device)."""
    return os.environ.get("SPMCTS_DIST_SINGLE", "0") == "1"


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's environment (no-op for world size 1 unless
    SPMCTS_DIST_SINGLE=1)."""
    rank, world, local = env_rank()
    if torch.cuda.is_available() and torch.cuda.device_count() > 0:
        local = local % torch.cuda.device_count()  # (rehearsals: several ranks on a 1-GPU box)
    if (world > 1 or single_rank_group()) and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("SPMCTS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if os.environ.get("SPMCTS_DIST_INIT"):  # e.g. file:///tmp/x (tests: no TCP port to race for)
            kw["init_method"] = os.environ["SPMCTS_DIST_INIT"]
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def local_device():
    """This rank's GPU (LOCAL_RANK, wrapped onto the visible devices)."""
    local = env_rank()[2]
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return torch.device("cuda", local % n) if n else torch.device("cpu")


def is_distributed():
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or single_rank_group())


def _comm_device():
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def barrier():
    if is_distributed():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_stats(stats):
    """Sum an int64 stats vector over ranks (returns a CPU tensor)."""
    t = torch.as_tensor(stats, dtype=torch.int64)
    if not is_distributed():
        return t.cpu()
    t = t.to(_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu()


def all_ranks_true(flag):
    """True iff `flag` holds on every rank (an all_reduce MIN; local value without a process group)."""
    if not is_distributed():
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def all_reduce_max(value):
    t = torch.tensor([float(value)], dtype=torch.float64)
    if not is_distributed():
        return float(t[0])
    t = t.to(_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.cpu()[0])


# ---------------------------------------------------------------- Move records
_FIELDS = (("state", torch.int8), ("tree_probs", torch.float32), ("q", torch.float64), ("q_f64", torch.uint8),
           ("z", torch.float32), ("game", torch.int64))


def pack_moves(moves):
    """Dict of per-record tensors -> uint8 [n, row_bytes] (one row per Move)."""
    n = moves["z"].shape[0]
    cols = []
    for name, dt in _FIELDS:
        t = moves[name].to(dt)
        per_row = 1
        for d in t.shape[1:]:
            per_row *= int(d)
        t = t.reshape(n, per_row).contiguous()  # explicit width: n may be 0
        cols.append(t.view(torch.uint8).reshape(n, per_row * t.element_size()))
    return torch.cat(cols, dim=1)


def unpack_moves(rows, cells, n_actions):
    """uint8 [n, row_bytes] -> dict of per-record tensors, on the rows' device."""
    widths = {"state": cells, "tree_probs": 4 * n_actions, "q": 8, "q_f64": 1, "z": 4, "game": 8}
    out, off = {}, 0
    for name, dt in _FIELDS:
        w = widths[name]
        chunk = torch.empty((rows.shape[0], w), dtype=torch.uint8, device=rows.device).copy_(rows[:, off:off + w])
        t = chunk.view(dt)
        out[name] = t if name in ("state", "tree_probs") else t.reshape(-1)
        off += w
    return out


def row_bytes(cells, n_actions):
    return cells + 4 * n_actions + 8 + 1 + 4 + 8


class MoveExchange:
    """Episode-batch exchange of Move records and statistics (rank `dst` owns the replay).

    `stage(moves)` is the engines' per-ply on_moves callback: without a process group it hands the
    records straight to `sink`; with one it only packs them into device rows (no collective, no
    host synchronisation).  `end_ply(stats_fn, done)` runs an exchange round every `every` plies
    (or when `force`): one all_gather of an int64 header [rows, not-done, stats...] per rank, then
    one gather of the rows padded to the largest count, to `dst` only.  On `dst` the rows are
    unpacked on the device and passed to `sink`.  It returns None on plies without a round, else
    (all ranks done, stats summed over ranks), so loops that end on it stay in step; in a single
    process every ply returns (done, stats) (end_ply).
    """

    def __init__(self, cells, n_actions, sink=None, every=8, dst=0):
        self.cells, self.A, self.sink, self.every, self.dst = cells, n_actions, sink, max(1, int(every)), dst
        self.width = row_bytes(cells, n_actions)
        self._staged = []
        self._plies = 0
        self.rounds = 0
        self.rows_gathered = 0
        self.seconds = 0.0  # host wall time spent in exchange rounds (this rank)

    def stage(self, moves):
        if not is_distributed():
            n = int(moves["z"].shape[0])
            self.rows_gathered += n
            if self.sink is not None and n:
                self.sink(moves)
            return
        if int(moves["z"].shape[0]):
            self._staged.append(pack_moves(moves))

    def end_ply(self, stats_fn=None, done=False, force=False):
        """Round plies (every `every`-th ply, or `force`) return (all ranks done, statistics summed over
        ranks); other plies return None under a process group.  In a single process there is nothing
        to exchange: every ply returns (done, stats), where stats is this process's statistics on
        round plies and None on the others (stats_fn reads device counters, so it is not called on
        every ply)."""
        self._plies += 1
        round_ply = force or self._plies % self.every == 0
        if not is_distributed():
            return bool(done), ([int(x) for x in stats_fn()] if stats_fn is not None and round_ply else None)
        if not round_ply:
            return None
        return self.exchange(stats_fn() if stats_fn is not None else [], done)

    def exchange(self, stats, done):
        t0 = time.perf_counter()
        try:
            return self._exchange(stats, done)
        finally:
            self.seconds += time.perf_counter() - t0

    def _exchange(self, stats, done):
        dev = _comm_device()
        world = dist.get_world_size()
        rows = torch.cat(self._staged, 0).to(dev) if self._staged else torch.zeros((0, self.width), dtype=torch.uint8,
                                                                                  device=dev)
        self._staged = []
        head = torch.tensor([rows.shape[0], 0 if done else 1] + [int(x) for x in stats], dtype=torch.int64, device=dev)
        heads = [torch.zeros_like(head) for _ in range(world)]
        dist.all_gather(heads, head)
        h = torch.stack(heads).cpu()
        counts = h[:, 0].tolist()
        all_done = int(h[:, 1].sum()) == 0
        mx = max(counts)
        if mx:
            pad = torch.zeros((mx, self.width), dtype=torch.uint8, device=dev)
            pad[: rows.shape[0]] = rows
            bufs = [torch.zeros_like(pad) for _ in range(world)] if dist.get_rank() == self.dst else None
            dist.gather(pad, gather_list=bufs, dst=self.dst)
            if bufs is not None:
                allrows = torch.cat([b[:c] for b, c in zip(bufs, counts) if c], 0)
                self.rows_gathered += int(allrows.shape[0])
                if self.sink is not None:
                    self.sink(unpack_moves(allrows, self.cells, self.A))
        self.rounds += 1
        return all_done, h[:, 2:].sum(0).tolist()


def broadcast_state_dict(module, src=0):
    """Epoch-boundary weight refresh from the trainer rank (in place): the whole state_dict in ONE
    flat buffer per dtype (float parameters / buffers; the int64 BatchNorm counters), i.e. one or
    two broadcasts per epoch instead of one per tensor."""
    if not is_distributed():
        return
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

    dev = _comm_device()
    groups = {}
    for t in module.state_dict().values():
        groups.setdefault(t.dtype, []).append(t)
    for dt in sorted(groups, key=str):  # the same order on every rank
        ts = groups[dt]
        flat = _flatten_dense_tensors([t.detach().reshape(-1) for t in ts]).to(dev)
        dist.broadcast(flat, src=src)
        with torch.no_grad():
            for t, v in zip(ts, _unflatten_dense_tensors(flat, [t.reshape(-1) for t in ts])):
                t.copy_(v.reshape(t.shape).to(t.device))


# ---------------------------------------------------------------- self-launch (one process per GPU)
def free_port():
    """A free TCP port on 127.0.0.1 for a local rendezvous."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    """torchrun's per-rank environment for a single-node job (MASTER_ADDR 127.0.0.1)."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def in_launched_job():
    """True when this process is already one rank of a launched job (torchrun or a self-launch)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def check_devices(n):
    """One process per GPU: refuse `n` ranks on fewer visible GPUs unless SPMCTS_ALLOW_OVERSUBSCRIBE=1
    (rehearsals of N ranks on a smaller box; RCCL refuses two ranks on one GPU, so such a rehearsal
    uses SPMCTS_DIST_BACKEND=gloo).  Counting devices does not initialise the GPU."""
    have = torch.cuda.device_count()
    if have < n and os.environ.get("SPMCTS_ALLOW_OVERSUBSCRIBE", "0") != "1":
        raise RuntimeError(f"{n} ranks requested (one per GPU) but only {have} GPU(s) are visible; set "
                           f"SPMCTS_ALLOW_OVERSUBSCRIBE=1 (with SPMCTS_DIST_BACKEND=gloo) to rehearse on fewer GPUs")
    return have


def assert_gpu_untouched(what):
    """launch_script's parent (bench.py --gpus N) only waits for its N rank processes: it must not have
    initialised HIP, or its own device context would sit on GPU 0 beside rank 0's for the whole job (and a
    GPU-initialised process may start children but never exec).  Raises RuntimeError if it has
    (torch.cuda.is_initialized(): device counting does not initialise, any allocation or kernel does).
    spawn_ranks (SelfPlayScheduler(gpus=N)) does not assert this: its parent keeps the caller's network and
    may have used the GPU before (a notebook, the GPU tests), and starting child processes from it is safe."""
    if torch.cuda.is_initialized():
        raise RuntimeError(f"{what}: this process has already initialised the GPU; start the rank processes "
                           f"before any GPU call (bench.py --gpus N and SelfPlayScheduler(gpus=N) do)")


def launch_script(argv, n, poll=0.2):
    """Run `python argv` as n ranks of a single-node job (bench.py --gpus N without torchrun): each
    child gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun would set them.  Must be called
    before this process touches the GPU (the children are started, never exec'd into).  If a rank
    fails, the others are stopped.  Returns the first non-zero exit code, else 0."""
    import subprocess
    import sys

    assert_gpu_untouched("launch_script")
    port = free_port()
    procs = [subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, n, port)) for r in range(n)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code and not rc:
                    rc = code
                    for q in procs:  # a lost rank would leave the others waiting in a collective
                        q.terminate()
            time.sleep(poll)
    finally:
        for p in procs:
            p.kill()
    return rc


def _spawned_rank(rank, world, port, fn, args, kwargs):
    os.environ.update(rank_env(rank, world, port, base={}))
    fn(*args, **kwargs)


def spawn_ranks(fn, n, *args, timeout=None, **kwargs):
    """Run fn(*args, **kwargs) in n fresh processes (spawn), rank r with torchrun's environment: how
    SelfPlayScheduler starts one process per GPU itself, as the reference's scheduler starts its
    own worker processes (self_play_parallel.py:95-171).  fn and its arguments must pickle; CPU
    tensors travel by shared memory.  The ranks are watched together: the first rank that exits
    non-zero gets the others terminated at once (a survivor would otherwise wait in a collective for
    the backend's timeout), and RuntimeError is raised.  `timeout` (seconds, None = none) bounds the
    whole run the same way."""
    import multiprocessing as mp
    from multiprocessing.connection import wait

    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_spawned_rank, args=(r, n, port, fn, args, kwargs)) for r in range(n)]
    for p in procs:
        p.start()
    failed = []
    t_end = None if timeout is None else time.monotonic() + timeout
    live = {p.sentinel: (r, p) for r, p in enumerate(procs)}
    try:
        while live:
            left = None if t_end is None else max(0.0, t_end - time.monotonic())
            ready = wait(list(live), timeout=left)
            if not ready:
                failed.append(("timeout", timeout))
                break
            for s in ready:
                r, p = live.pop(s)
                p.join()
                if p.exitcode:
                    failed.append((r, p.exitcode))
            if failed:
                break
    finally:
        for r, p in enumerate(procs):
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    if failed:
        raise RuntimeError(f"rank process(es) failed: {failed}")


def rank_report(values):
    """All-gather one float64 vector per rank (every rank gets the [world, len] table; a one-row
    table without a process group): the per-rank lines of bench.py's N-rank report (positions/s,
    timed seconds, exchange rounds and their cost), so a scaling record shows stragglers directly."""
    t = torch.as_tensor([float(x) for x in values], dtype=torch.float64)
    if not is_distributed():
        return [t.tolist()]
    dev = _comm_device()
    t = t.to(dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]
