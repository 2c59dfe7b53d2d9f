"""Python handle on one device arena (include/spmcts.h) — torch tensors in, torch tensors out.

All buffers handed to the library are torch tensors on the arena's device; the
library launches on `torch.cuda.current_stream()` of that device, so the
network that consumes the leaf rows runs on the same stream with no extra
synchronisation.  The only host round trip per simulation is reading the
number of leaf rows (`select()` returns it as a Python int).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

GAMES = {"connect4": (_lib.CONNECT4, 7, 6, 7), "tictactoe": (_lib.TICTACTOE, 3, 3, 9)}
LEAF_FORMATS = {"f32": _lib.LEAF_F32, "f16": _lib.LEAF_F16, "bf16": _lib.LEAF_BF16, "board": _lib.LEAF_BOARD_I64}
_LEAF_DTYPES = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16, "board": torch.int64}


def game_of_env(env):
    """Map a reference-style env (class or instance) to an arena game name.

    Accepts this package's envs and the reference's Connect4Env / TicTacToeEnv
    (games/connect4/connect4env.py, games/tictactoe/tictactoe_env.py) by shape.
    """
    e = env() if isinstance(env, type) else env
    name = type(e).__name__.lower()
    w, h = getattr(e, "width", None), getattr(e, "height", None)
    n = e.action_space.n if hasattr(e, "action_space") else getattr(e, "n_actions", None)
    if "connect4" in name or (w, h, n) == (7, 6, 7):
        game = "connect4"
    elif "tictactoe" in name or (w, h, n) == (3, 3, 9):
        game = "tictactoe"
    else:
        raise ValueError(f"unsupported environment {type(e).__name__}")
    gid, W, H, A = GAMES[game]
    if (w, h) != (W, H):
        raise ValueError(f"{game} arena is instantiated for {W}x{H} boards only, got {w}x{h}")
    return game


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Arena:
    """A device-resident forest of MCTS trees (+ optional self-play game slots)."""

    def __init__(self, game="connect4", n_trees=2, n_games=0, iterations=100, rng="philox", seed=0,
                 subsequence0=0, strong_play=False, evaluate=False, leaf_format="bf16", leaf_layout="nchw",
                 cpuct=4.0, x_noise=0.25, alpha=1.0, blocks_per_tree=0, device=None, search_threads=1):
        if not torch.cuda.is_available():
            raise _lib.SpmctsError("the HIP arena needs a GPU (torch.cuda.is_available() is False)")
        gid, W, H, A = GAMES[game]
        self.game, self.W, self.H, self.A = game, W, H, A
        self.cells = W * H
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.n_trees, self.n_games = n_trees, n_games
        self.leaf_format, self.leaf_layout = leaf_format, leaf_layout
        cfg = _lib.Config()
        cfg.game, cfg.width, cfg.height = gid, W, H
        cfg.n_trees, cfg.n_games, cfg.iterations = n_trees, n_games, iterations
        cfg.blocks_per_tree = blocks_per_tree
        cfg.rng_mode = _lib.RNG_TAPE if rng == "tape" else _lib.RNG_PHILOX
        cfg.strong_play, cfg.evaluate = int(bool(strong_play)), int(bool(evaluate))
        cfg.leaf_format = LEAF_FORMATS[leaf_format]
        cfg.leaf_layout = _lib.NHWC if leaf_layout == "nhwc" else _lib.NCHW
        cfg.compact = 1
        # K simulations in flight per tree with virtual loss (mcts.py:328-331); rows = n_trees * K
        self.search_threads = K = max(1, int(search_threads))
        cfg.search_threads = K
        cfg.cpuct, cfg.x_noise, cfg.alpha = float(cpuct), float(x_noise), float(alpha)
        cfg.seed, cfg.subsequence0 = int(seed) & (2**64 - 1), int(subsequence0)
        self.cfg = cfg
        L = _lib.lib()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("spmcts_arena_create", ctypes.byref(cfg), self.device.index, ctypes.byref(h))
        self.h = h
        geo = [ctypes.c_int32() for _ in range(6)]
        call("spmcts_arena_geometry", h, *[ctypes.byref(g) for g in geo])
        self.blocks_per_tree = geo[3].value
        dev = self.device
        rows = max(n_trees * K, n_games, 1)
        self.max_rows = rows
        if leaf_format == "board":
            self._leaves = torch.zeros((rows, W, H), dtype=torch.int64, device=dev)
        elif leaf_layout == "nhwc":
            self._leaves = torch.zeros((rows, W, H, 3), dtype=_LEAF_DTYPES[leaf_format], device=dev)
        else:
            self._leaves = torch.zeros((rows, 3, W, H), dtype=_LEAF_DTYPES[leaf_format], device=dev)
        self._count = torch.zeros(4, dtype=torch.int32, device=dev)
        self._count_host = torch.zeros(4, dtype=torch.int32).pin_memory()
        self._finish = torch.zeros(2, dtype=torch.int32, device=dev)
        self._i32 = torch.zeros(rows, dtype=torch.int32, device=dev)
        self._i8 = torch.zeros(rows, dtype=torch.int8, device=dev)
        self.n_active = 0
        self.seg1 = n_trees * K  # first leaf row of network 1 (two-network arenas)
        self._L = L

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            _lib.lib().spmcts_arena_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ helpers
    def _dev_i32(self, xs):
        return torch.as_tensor(np.asarray(xs, dtype=np.int32)).to(self.device)

    def _dev_i8(self, xs):
        return torch.as_tensor(np.asarray(xs, dtype=np.int8)).to(self.device)

    def leaves(self, n):
        """Leaf rows [:n] as the network's input tensor ([n, 3, W, H]; channels_last if NHWC)."""
        x = self._leaves[:n]
        if self.leaf_format != "board" and self.leaf_layout == "nhwc":
            x = x.permute(0, 3, 1, 2)  # NCHW view with channels_last strides
        return x

    def leaves_from(self, row0, n):
        """Leaf rows [row0, row0 + n) (network-1 rows start at `seg1`)."""
        x = self._leaves[row0:row0 + n]
        if self.leaf_format != "board" and self.leaf_layout == "nhwc":
            x = x.permute(0, 3, 1, 2)
        return x

    def _read_count(self):
        self._count_host.copy_(self._count, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return int(self._count_host[0])

    def segment_counts(self):
        """(network-0 rows, network-1 rows) of the last select / play_action / games_end_ply (sync)."""
        self._count_host.copy_(self._count, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return int(self._count_host[1]), int(self._count_host[2])

    # ------------------------------------------------------------------ configuration
    def set_root_prior(self, probs, net=0):
        p = torch.as_tensor(probs, dtype=torch.float32).to(self.device).contiguous()
        if net == 0:
            self._root_prior = p
            call("spmcts_set_root_prior", self.h, ptr(p), _stream())
        else:
            self._root_prior1 = p
            call("spmcts_set_root_prior_net", self.h, int(net), ptr(p), _stream())

    def set_tree_players(self, nets=None, kinds=None, budgets=None):
        """Per-tree network id (0/1), player kind (_lib.PLAYER_*) and simulations per search.

        Network-1 leaves are written from row `seg1` (= number of network-0 trees) on."""
        T = self.n_trees

        def arr(x, ctype, dtype):
            if x is None:
                return None
            a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
            if a.shape != (T,):
                raise ValueError(f"expected {T} per-tree entries, got {a.shape}")
            return a.ctypes.data_as(ctypes.POINTER(ctype)), a

        n = arr(nets, ctypes.c_uint8, np.uint8)
        k = arr(kinds, ctypes.c_uint8, np.uint8)
        b = arr(budgets, ctypes.c_int32, np.int32)
        torch.cuda.current_stream().synchronize()
        call("spmcts_set_tree_players", self.h, n[0] if n else None, k[0] if k else None, b[0] if b else None)
        seg = ctypes.c_int32()
        call("spmcts_arena_segments", self.h, ctypes.byref(seg))
        self.seg1 = seg.value

    def set_tree_search(self, alpha=None, strong_play=None, search_threads=None):
        """Per-tree search settings (include/spmcts.h spmcts_set_tree_search): each side of an
        evaluation game searches with its own MCTreeSearch kwargs (selfplayworker.py:71-81):
        Dirichlet alpha, strong_play, sims in flight (1 .. this arena's search_threads).  None =
        unchanged."""
        T = self.n_trees

        def arr(x, ctype, dtype):
            if x is None:
                return None
            a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
            if a.shape != (T,):
                raise ValueError(f"expected {T} per-tree entries, got {a.shape}")
            return a.ctypes.data_as(ctypes.POINTER(ctype)), a

        al = arr(alpha, ctypes.c_double, np.float64)
        st = arr(strong_play, ctypes.c_uint8, np.uint8)
        k = arr(search_threads, ctypes.c_int32, np.int32)
        torch.cuda.current_stream().synchronize()
        call("spmcts_set_tree_search", self.h, al[0] if al else None, st[0] if st else None, k[0] if k else None)
        if search_threads is not None:
            self.tree_threads = np.asarray(search_threads, dtype=np.int64)

    def games_set_record(self, record=True):
        call("spmcts_games_set_record", self.h, int(bool(record)))

    def set_leaf_dedup(self, on=True):
        """One leaf row per distinct network input of a simulation step (search_threads > 1;
        include/spmcts.h spmcts_set_leaf_dedup).  Only for evaluators that are a pure function of the
        leaf planes (the ResNet evaluators), not for per-row salted table nets."""
        call("spmcts_set_leaf_dedup", self.h, int(bool(on)))
        self.leaf_dedup = bool(on) and self.search_threads > 1

    def set_leaf_peer(self, leader):
        """Cross-lane leaf dedup (include/spmcts.h spmcts_set_leaf_peer): in each simulation step a pending leaf
        whose network input `leader` (another lane's arena, stepped first) evaluates in the same step takes the
        leader's row.  The follower's simulation-step expand is then preceded by peer_push.  None unpairs."""
        call("spmcts_set_leaf_peer", self.h, None if leader is None else leader.h)
        self._leader = leader  # the leader outlives the pairing (its destroy unpairs its followers)

    def peer_push(self, probs, values, leader_probs, leader_values, leader_stream):
        """Before expand() of a follower lane's simulation step: the leader's outputs of the step (its
        evaluator's output buffers, valid on `leader_stream`) fill the leader-served rows of probs / values."""
        assert probs.dtype == torch.float32 and probs.is_contiguous() and values.is_contiguous()
        assert leader_probs.dtype == torch.float32 and leader_probs.is_contiguous() and leader_values.is_contiguous()
        call("spmcts_peer_push", self.h, ptr(probs), ptr(values), ptr(leader_probs), ptr(leader_values), _stream(),
             ctypes.c_void_p(leader_stream.cuda_stream))

    def set_eval_cache(self, window, capacity_log2=0):
        """Evaluation cache (include/spmcts.h spmcts_set_eval_cache): a leaf whose network input this arena
        evaluated in the last `window` plies (searches) takes those outputs instead of a row of its own; 0 =
        off.  Needs leaf dedup (idle without it).  Same evaluator contract as leaf dedup (pure,
        batch-independent; the two networks of an evaluation arena keep separate keys); call eval_cache_clear()
        when the weights change."""
        torch.cuda.current_stream().synchronize()
        call("spmcts_set_eval_cache", self.h, int(window), int(capacity_log2))
        self.eval_cache = int(window)

    def eval_cache_clear(self):
        call("spmcts_eval_cache_clear", self.h)

    def set_tapes(self, tapes):
        """Parity mode: one flat float64 stream per tree (list indexed by tree id)."""
        offs = np.zeros(self.n_trees + 1, dtype=np.int64)
        for t in range(self.n_trees):
            offs[t + 1] = offs[t] + (len(tapes[t]) if t < len(tapes) and tapes[t] is not None else 0)
        flat = np.concatenate([np.asarray(tapes[t], dtype=np.float64) for t in range(min(len(tapes), self.n_trees))
                               if tapes[t] is not None] + [np.zeros(1)])
        self._tape = torch.as_tensor(flat).to(self.device)
        self._tape_offs = torch.as_tensor(offs).to(self.device)
        call("spmcts_set_tape", self.h, ptr(self._tape), ptr(self._tape_offs), _stream())

    # ------------------------------------------------------------------ tree API
    def tree_reset(self, trees, players, priors=None):
        """priors: optional float32 [n, A] per-tree root priors (default: the arena's root prior)."""
        t = self._dev_i32(trees)
        p = self._dev_i8(players)
        pr = None if priors is None else torch.as_tensor(priors, dtype=torch.float32).to(self.device).contiguous()
        call("spmcts_tree_reset", self.h, ptr(t), ptr(p), ptr(pr), len(trees), _stream())

    def search_begin(self, trees):
        t = self._dev_i32(trees)
        self._active = t
        self.n_active = len(trees)
        call("spmcts_search_begin", self.h, ptr(t), len(trees), _stream())

    def select(self, timer=None):
        """One simulation for every active tree; returns the number of leaf rows to evaluate.

        `timer` (optional): object with start()/stop() bracketing the tree-walk kernel alone
        (HIP events on this stream, used by bench.py for the select roofline)."""
        if timer is None:
            call("spmcts_select", self.h, ptr(self._leaves), ptr(self._count), _stream())
        else:
            timer.start()
            call("spmcts_select_tree", self.h, _stream())
            timer.stop()
            call("spmcts_leaf_rows", self.h, ptr(self._leaves), ptr(self._count), _stream())
        return self._read_count()

    def select_async(self, timer=None):
        """select() without reading the row count back (for device-count evaluators)."""
        if timer is None:
            call("spmcts_select", self.h, ptr(self._leaves), ptr(self._count), _stream())
        else:
            timer.start()
            call("spmcts_select_tree", self.h, _stream())
            timer.stop()
            call("spmcts_leaf_rows", self.h, ptr(self._leaves), ptr(self._count), _stream())

    def leaf_rows_async(self):
        """Gather the pending leaves into network rows (k_scan_need + k_encode) without a select."""
        call("spmcts_leaf_rows", self.h, ptr(self._leaves), ptr(self._count), _stream())

    def games_end_ply_async(self):
        call("spmcts_games_end_ply", self.h, ptr(self._leaves), ptr(self._count), _stream())

    @property
    def count_dev(self):
        """Device int32 holding the row count of the last select / play_action / games_end_ply."""
        return self._count

    def segment_count_dev(self, net):
        """Device int32 holding network `net`'s row count (element 1 + net of the count buffer)."""
        return self._count[1 + net:2 + net]

    def expand(self, probs, values):
        probs = probs.float().contiguous()
        values = values.float().reshape(-1).contiguous()
        call("spmcts_expand", self.h, ptr(probs), ptr(values), _stream())

    def expand2(self, probs0, values0, probs1, values1):
        """Two-network expand: network-0 outputs by row, network-1 outputs by row - seg1."""
        t = [x.float().contiguous() if x.dtype != torch.float32 or not x.is_contiguous() else x
             for x in (probs0, values0.reshape(-1), probs1, values1.reshape(-1))]
        call("spmcts_expand2", self.h, *[ptr(x) for x in t], _stream())

    def search_end(self, temp=1.0):
        n = self.n_active
        dev = self.device
        out = dict(
            action=torch.zeros(n, dtype=torch.int32, device=dev),
            state=torch.zeros((n, self.cells), dtype=torch.int8, device=dev),
            tree_probs=torch.zeros((n, self.A), dtype=torch.float32, device=dev),
            q=torch.zeros(n, dtype=torch.float64, device=dev),
            q_f64=torch.zeros(n, dtype=torch.uint8, device=dev),
            recorded=torch.zeros(n, dtype=torch.uint8, device=dev),
        )
        call("spmcts_search_end", self.h, float(temp), ptr(out["action"]), ptr(out["state"]), ptr(out["tree_probs"]),
             ptr(out["q"]), ptr(out["q_f64"]), ptr(out["recorded"]), _stream())
        return out

    def play_action(self, trees, actions):
        t = self._dev_i32(trees)
        a = self._dev_i32(actions)
        call("spmcts_play_action", self.h, ptr(t), ptr(a), len(trees), ptr(self._leaves), ptr(self._count), _stream())
        return self._read_count()

    def leaf_trees(self, n):
        """Tree id of each of the first n leaf rows (device int32 tensor)."""
        out = torch.empty(self.n_trees * self.search_threads, dtype=torch.int32, device=self.device)
        call("spmcts_leaf_trees", self.h, ptr(out), _stream())
        out = out[:n]
        return out // self.search_threads if self.search_threads > 1 else out

    def root_stats(self, tree):
        A, cells = self.A, self.cells
        cn = (ctypes.c_int32 * A)()
        cw = (ctypes.c_double * A)()
        cp = (ctypes.c_float * A)()
        rn, rw, rp = ctypes.c_int32(), ctypes.c_double(), ctypes.c_int32()
        board = (ctypes.c_int8 * cells)()
        torch.cuda.current_stream().synchronize()
        call("spmcts_root_stats", self.h, int(tree), cn, cw, cp, ctypes.byref(rn), ctypes.byref(rw), ctypes.byref(rp),
             board)
        return dict(child_n=list(cn), child_w=list(cw), child_p=list(cp), root_n=rn.value, root_w=rw.value,
                    root_player=rp.value, board=np.array(list(board), dtype=np.int8).reshape(self.W, self.H))

    # ------------------------------------------------------------------ games API
    def games_start(self, slots, priors=None):
        """priors: optional float32 [n, 2, A] (policy tree, opponent tree) root priors per game."""
        s = self._dev_i32(slots)
        pr = None if priors is None else torch.as_tensor(priors, dtype=torch.float32).to(self.device).contiguous()
        call("spmcts_games_start", self.h, ptr(s), ptr(pr), len(slots), _stream())

    def games_set_limit(self, max_games):
        torch.cuda.current_stream().synchronize()
        call("spmcts_games_set_limit", self.h, int(max_games))

    def games_begin_ply(self):
        self.n_active = self.n_games
        call("spmcts_games_begin_ply", self.h, _stream())

    def games_end_ply(self):
        call("spmcts_games_end_ply", self.h, ptr(self._leaves), ptr(self._count), _stream())
        return self._read_count()

    def games_finish_ply(self, refill=True):
        call("spmcts_games_finish_ply", self.h, int(bool(refill)), ptr(self._finish), _stream())
        f = self._finish.cpu()
        return int(f[0]), int(f[1])

    def finish_export_async(self, refill=True):
        """games_finish_ply + export_moves of the whole export ring without a host synchronisation: the records go
        to persistent buffers of the ring's capacity and the counts to pinned host memory; returns an event for
        finish_export_result.  Several lanes can queue theirs before the host waits on any of them."""
        if getattr(self, "_exp", None) is None:
            cap = max(64, 4 * self.n_games * ((self.cells + 1) // 2 + 1))  # spmcts.hip plan_arena: ex_cap (MAXM)
            dev = self.device
            self._exp = dict(
                state=torch.empty((cap, self.cells), dtype=torch.int8, device=dev),
                tree_probs=torch.empty((cap, self.A), dtype=torch.float32, device=dev),
                q=torch.empty(cap, dtype=torch.float64, device=dev),
                q_f64=torch.empty(cap, dtype=torch.uint8, device=dev),
                z=torch.empty(cap, dtype=torch.float32, device=dev),
                game=torch.empty(cap, dtype=torch.int64, device=dev),
            )
            self._exp_cap = cap
            self._exp_count = torch.zeros(4, dtype=torch.int32, device=dev)
            self._exp_host = torch.zeros(3, dtype=torch.int32).pin_memory()
        e = self._exp
        call("spmcts_games_finish_ply", self.h, int(bool(refill)), ptr(self._finish), _stream())
        call("spmcts_export_moves", self.h, ptr(e["state"]), ptr(e["tree_probs"]), ptr(e["q"]), ptr(e["q_f64"]),
             ptr(e["z"]), ptr(e["game"]), self._exp_cap, ptr(self._exp_count), _stream())
        self._exp_host[0:2].copy_(self._finish, non_blocking=True)
        self._exp_host[2:3].copy_(self._exp_count[0:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def finish_export_result(self, ev):
        """(#games finished, Move records) of finish_export_async once `ev` has completed (waits for it); the
        records are copies (queued on the current stream), so the persistent buffers can be reused next ply."""
        ev.synchronize()
        finished, ring, k = (int(x) for x in self._exp_host.tolist())
        if k != ring:
            raise _lib.SpmctsError(f"Move export took {k} of {ring} ring records (buffer capacity {self._exp_cap})")
        moves = {key: v[:k].clone() for key, v in self._exp.items()} if k else None
        return finished, moves

    def export_moves(self, max_records):
        dev = self.device
        n = max(1, int(max_records))
        out = dict(
            state=torch.zeros((n, self.cells), dtype=torch.int8, device=dev),
            tree_probs=torch.zeros((n, self.A), dtype=torch.float32, device=dev),
            q=torch.zeros(n, dtype=torch.float64, device=dev),
            q_f64=torch.zeros(n, dtype=torch.uint8, device=dev),
            z=torch.zeros(n, dtype=torch.float32, device=dev),
            game=torch.zeros(n, dtype=torch.int64, device=dev),
        )
        call("spmcts_export_moves", self.h, ptr(out["state"]), ptr(out["tree_probs"]), ptr(out["q"]),
             ptr(out["q_f64"]), ptr(out["z"]), ptr(out["game"]), n, ptr(self._count), _stream())
        k = self._read_count()
        return {key: v[:k] for key, v in out.items()}

    def games_state(self):
        G = self.n_games
        active = (ctypes.c_uint8 * G)()
        ply = (ctypes.c_int32 * G)()
        swap = (ctypes.c_uint8 * G)()
        gid = (ctypes.c_int64 * G)()
        torch.cuda.current_stream().synchronize()
        call("spmcts_games_state", self.h, active, ply, swap, gid)
        return dict(state=np.array(list(active)), ply=np.array(list(ply)), swap=np.array(list(swap)),
                    game_id=np.array(list(gid)))

    # ------------------------------------------------------------------ diagnostics
    def counters(self):
        c = _lib.Counters()
        torch.cuda.current_stream().synchronize()
        call("spmcts_get_counters", self.h, ctypes.byref(c))
        return c.as_dict()

    def check(self):
        torch.cuda.current_stream().synchronize()
        rc = _lib.lib().spmcts_check(self.h)
        if rc != 0:
            c = self.counters()
            raise _lib.SpmctsError(f"arena device error: {_lib.describe_flags(c['error_flags'])}")


def table_net_eval(game, leaves, leaf_format, leaf_layout, salt=0, salts=None):
    """Run the deterministic table network kernel over leaf rows (parity tests / smoke).

    `salts` (int64 tensor [n] on the device, optional) gives every row its own network."""
    gid, W, H, A = GAMES[game]
    n = leaves.shape[0]
    dev = leaves.device
    probs = torch.empty((max(n, 1), A), dtype=torch.float32, device=dev)
    values = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    if n:
        src = leaves
        if leaf_format != "board" and leaf_layout == "nhwc":
            src = leaves.permute(0, 2, 3, 1)  # back to the NHWC storage order
        call("spmcts_table_net", gid, W, H, ptr(src), LEAF_FORMATS[leaf_format],
             _lib.NHWC if leaf_layout == "nhwc" else _lib.NCHW, n, int(salt) & (2**64 - 1),
             ptr(salts) if salts is not None else None, ptr(probs), ptr(values), _stream())
    return probs[:n], values[:n]
