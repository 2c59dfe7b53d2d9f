"""ctypes binding of the HIP arena library (include/spmcts.h).

The library is built in-tree by `__graft_entry__.build()` / `make -C
self_play_reinforcement_learning_amd/csrc` into
`self_play_reinforcement_learning_amd/libspmcts.so`.  There is deliberately
no fallback: if the library is missing, loading raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "libspmcts.so")
LIB_PATH = os.environ.get("SPMCTS_LIB", _DEFAULT_LIB)

CONNECT4, TICTACTOE = 0, 1
RNG_PHILOX, RNG_TAPE = 0, 1
TOWER_PACK = 1  # spmcts_tower_forward_dev flags (include/spmcts.h SPMCTS_TOWER_PACK)
TOWER_F16 = 2  # fp16 weights / activations / head features (include/spmcts.h SPMCTS_TOWER_F16)
LEAF_F32, LEAF_F16, LEAF_BF16, LEAF_BOARD_I64 = 0, 1, 2, 3
WLAYOUT_32X32, WLAYOUT_M16 = 0, 1  # spmcts_tower_weight_layout (include/spmcts.h SPMCTS_WLAYOUT_*)
NCHW, NHWC = 0, 1
PLAYER_MCTS, PLAYER_RANDOM, PLAYER_LOOKAHEAD = 0, 1, 2

ERR_FLAGS = {
    0x1: "node pool exhausted",
    0x2: "RNG tape exhausted",
    0x4: "select reached a node without valid children",
    0x8: "illegal action",
    0x10: "inconsistent tree state",
    0x20: "move export ring overflow",
}


class Config(ctypes.Structure):
    _fields_ = [
        ("game", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("n_trees", ctypes.c_int32),
        ("n_games", ctypes.c_int32),
        ("iterations", ctypes.c_int32),
        ("blocks_per_tree", ctypes.c_int32),
        ("rng_mode", ctypes.c_int32),
        ("strong_play", ctypes.c_int32),
        ("evaluate", ctypes.c_int32),
        ("leaf_format", ctypes.c_int32),
        ("leaf_layout", ctypes.c_int32),
        ("compact", ctypes.c_int32),
        ("search_threads", ctypes.c_int32),
        ("cpuct", ctypes.c_double),
        ("x_noise", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("subsequence0", ctypes.c_uint64),
    ]


class Counters(ctypes.Structure):
    _fields_ = [
        ("sims", ctypes.c_int64),
        ("nn_leaves", ctypes.c_int64),
        ("terminal_leaves", ctypes.c_int64),
        ("depth_sum", ctypes.c_int64),
        ("set_node_expansions", ctypes.c_int64),
        ("moves", ctypes.c_int64),
        ("games_finished", ctypes.c_int64),
        ("positions_exported", ctypes.c_int64),
        ("results", (ctypes.c_int64 * 3) * 2),
        ("blocks_in_use_max", ctypes.c_int64),
        ("error_flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("leaked_sims", ctypes.c_int64),
        ("compactions", ctypes.c_int64),
        ("nn_rows", ctypes.c_int64),
        ("cache_rows", ctypes.c_int64),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("results", "reserved")}
        d["results"] = [[self.results[i][j] for j in range(3)] for i in range(2)]
        return d


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_D = ctypes.c_double

# name -> argtypes (restype is c_int for all)
_SIGS = {
    "spmcts_version": [],
    "spmcts_arena_bytes": [ctypes.POINTER(Config), ctypes.POINTER(_U64)],
    "spmcts_arena_create": [ctypes.POINTER(Config), ctypes.c_int, ctypes.POINTER(_P)],
    "spmcts_arena_destroy": [_P],
    "spmcts_arena_geometry": [_P] + [ctypes.POINTER(_I32)] * 6,
    "spmcts_set_root_prior": [_P, _P, _P],
    "spmcts_set_tape": [_P, _P, _P, _P],
    "spmcts_tree_reset": [_P, _P, _P, _P, _I32, _P],
    "spmcts_search_begin": [_P, _P, _I32, _P],
    "spmcts_select": [_P, _P, _P, _P],
    "spmcts_select_tree": [_P, _P],
    "spmcts_leaf_rows": [_P, _P, _P, _P],
    "spmcts_expand": [_P, _P, _P, _P],
    "spmcts_expand2": [_P, _P, _P, _P, _P, _P],
    "spmcts_set_tree_players": [_P, _P, _P, _P],
    "spmcts_set_tree_search": [_P, _P, _P, _P],
    "spmcts_arena_segments": [_P, ctypes.POINTER(_I32)],
    "spmcts_set_root_prior_net": [_P, _I32, _P, _P],
    "spmcts_games_set_record": [_P, _I32],
    "spmcts_search_end": [_P, _D, _P, _P, _P, _P, _P, _P, _P],
    "spmcts_play_action": [_P, _P, _P, _I32, _P, _P, _P],
    "spmcts_root_stats": [_P, _I32, _P, _P, _P, _P, _P, _P, _P],
    "spmcts_games_start": [_P, _P, _P, _I32, _P],
    "spmcts_games_set_limit": [_P, _I64],
    "spmcts_games_begin_ply": [_P, _P],
    "spmcts_games_end_ply": [_P, _P, _P, _P],
    "spmcts_games_finish_ply": [_P, _I32, _P, _P],
    "spmcts_export_moves": [_P, _P, _P, _P, _P, _P, _P, _I32, _P, _P],
    "spmcts_games_state": [_P, _P, _P, _P, _P],
    "spmcts_get_counters": [_P, ctypes.POINTER(Counters)],
    "spmcts_check": [_P],
    "spmcts_env_step": [_I32, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P],
    "spmcts_env_step_host": [_I32, _I32, _I32, _P, _I32, _I32, ctypes.POINTER(_I32), ctypes.POINTER(_I32)],
    "spmcts_valid_moves_host": [_I32, _I32, _I32, _P, _P],
    "spmcts_table_net": [_I32, _I32, _I32, _P, _I32, _I32, _I32, _U64, _P, _P, _P, _P],
    "spmcts_set_leaf_dedup": [_P, _I32],
    "spmcts_set_leaf_peer": [_P, _P],
    "spmcts_peer_push": [_P, _P, _P, _P, _P, _P, _P],
    "spmcts_set_eval_cache": [_P, _I32, _I32],
    "spmcts_eval_cache_clear": [_P],
    "spmcts_leaf_trees": [_P, _P, _P],
    "spmcts_copy_probe": [_P, _P, _U64, _P],
    "spmcts_conv3x3_supported": [_I32, _I32, _I32, _I32],
    "spmcts_conv3x3_pack": [_I32, _I32, _P, _P, _P, _P],
    "spmcts_conv3x3_fwd": [_I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P],
    "spmcts_conv3x3_wgrad": [_I32, _I32, _I32, _I32, _I32, _P, _P, _P, _I32, _P, _P, _P],
    "spmcts_tower_forward": [_I32, _I32, _I32, _I32, _P, _I32, _P, _P, _P, _I32, _P],
    "spmcts_tower_supported": [_I32, _I32, _I32],
    "spmcts_tower_weight_layout": [_I32, _I32, _I32],
    "spmcts_tower_heads": [_I32, _I32, _I32, _I32, _P, _I32, _P, _P, _P, _P, _I32, _P],
    "spmcts_head_epilogue": [_I32, _I32, _P, _I32, _I32, _P, _P, _P, _P],
    "spmcts_tower_forward_dev": [_I32, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _P, _I32, _P],
    "spmcts_tower_heads_dev": [_I32, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _P, _P, _I32, _P],
}

# every symbol the header declares (tests check the .so exports exactly these)
HEADER_SYMBOLS = sorted(list(_SIGS) + ["spmcts_last_error"])

_lib = None


class SpmctsError(RuntimeError):
    pass


def lib():
    """Load libspmcts.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SpmctsError(
                f"HIP arena library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C self_play_reinforcement_learning_amd/csrc`"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                # a build from before this entry point existed (SPMCTS_LIB pointing at an earlier library for a
                # same-box A/B): only the entry points it has are bound; the product library exports every
                # symbol the header declares (tests/test_native_lib.py)
                if os.path.realpath(LIB_PATH) == os.path.realpath(_DEFAULT_LIB):
                    raise
                continue
            f.argtypes = args
            f.restype = ctypes.c_int
        L.spmcts_last_error.argtypes = []
        L.spmcts_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


# environment switches read only by the A/B library (libspmcts_ab.so); the product library refuses them with
# SPMCTS_ERR_AB_SWITCH (-5, include/spmcts.h) rather than silently ignoring them
AB_SWITCHES = ("SPMCTS_TOWER_CG", "SPMCTS_TOWER_RING", "SPMCTS_TOWER_C256", "SPMCTS_WIDE_TAILS", "SPMCTS_HEADS",
               "SPMCTS_HEADS_C256", "SPMCTS_TREE_BLOCK", "SPMCTS_EXPAND_CO", "SPMCTS_TOWER_M16",
               "SPMCTS_TREE_COPIES", "SPMCTS_PEER_PUSH", "SPMCTS_CACHE_SHARE")
ERR_AB_SWITCH = -5


def tower_error(what, rc):
    """The SpmctsError of a failed tower entry point; -5 names the A/B switch that caused it."""
    if rc == ERR_AB_SWITCH:
        set_ = [n for n in AB_SWITCHES if n in os.environ]
        return SpmctsError(f"{what} failed ({rc}): {', '.join(set_) or 'an A/B switch'} is set, a switch of the A/B "
                           f"library (make ab: libspmcts_ab.so, SPMCTS_LIB=...); unset it to use the product library")
    return SpmctsError(f"{what} failed ({rc})")


def check(rc, what=""):
    if rc != 0:
        msg = lib().spmcts_last_error().decode(errors="replace")
        raise SpmctsError(f"{what} failed ({rc}): {msg}")
    return rc


def call(name, *args):
    return check(getattr(lib(), name)(*args), name)


def ptr(t):
    """Device/host pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def describe_flags(flags):
    return ", ".join(msg for bit, msg in ERR_FLAGS.items() if flags & bit) or "none"
