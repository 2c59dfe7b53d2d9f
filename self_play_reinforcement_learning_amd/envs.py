"""Board environments with the reference API (games/general/base_env.py:8-50).

`Connect4Env` (games/connect4/connect4env.py) and `TicTacToeEnv`
(games/tictactoe/tictactoe_env.py): int64 [W, H] boards indexed
[column, row], `step(action, player) -> (board, reward, done, info)`,
`valid_moves()`, `reset()`, `set_state()`, `max_moves()`, `action_space.n`,
callable clone.  `step` runs the same bitboard rules the HIP kernels use
(csrc/board.h), compiled for the host inside libspmcts.so — these objects are
for driving single games (manual play, tests, evaluation opponents); the
self-play hot path never calls them.
"""
import copy

import numpy as np

from . import _lib


class GameOver(Exception):
    pass


class Discrete:
    """gym.spaces.Discrete stand-in (only `.n` is used by the reference)."""

    def __init__(self, n):
        self.n = int(n)


class BaseEnv:
    def __call__(self):
        return copy.deepcopy(self)

    def num_actions(self):
        return self.action_space.n


class _BitboardEnv(BaseEnv):
    GAME = None

    def __init__(self, width, height, n_actions):
        self.width, self.height = width, height
        self.action_space = Discrete(n_actions)
        self.episode_over = False
        self.board = np.zeros([width, height], dtype=np.int64)

    def max_moves(self):
        return self.width * self.height

    def reset(self):
        self.episode_over = False
        self.board = np.zeros([self.width, self.height], dtype=np.int64)
        return self.board

    def set_state(self, state):
        self.board = state

    def get_state(self):
        return self.board, None

    def valid_moves(self):
        b = np.ascontiguousarray(self.board, dtype=np.int8)
        out = np.zeros(self.action_space.n, dtype=np.uint8)
        _lib.call("spmcts_valid_moves_host", self.GAME, self.width, self.height, b.ctypes.data_as(_lib.ctypes.c_void_p),
                  out.ctypes.data_as(_lib.ctypes.c_void_p))
        return out.astype(bool)

    def step(self, action, player=1):
        if self.episode_over:
            raise GameOver
        b = np.ascontiguousarray(self.board, dtype=np.int8)
        r = _lib.ctypes.c_int32()
        d = _lib.ctypes.c_int32()
        st = _lib.lib().spmcts_env_step_host(self.GAME, self.width, self.height, b.ctypes.data_as(_lib.ctypes.c_void_p),
                                             int(action), int(player), _lib.ctypes.byref(r), _lib.ctypes.byref(d))
        if st < 0:
            _lib.check(st, "env step")
        if st == 1:
            raise ValueError("column is full")
        self.board[...] = b.astype(np.int64)
        self.episode_over = bool(d.value)
        return self.board, int(r.value), self.episode_over, self._info()

    def _info(self):
        return None

    def render(self, board=None):
        board = self.board if board is None else board
        sym = {0: " ", 1: "X", -1: "O"}
        rows = ["|" + "|".join(sym[int(board[x, y])] for x in range(self.width)) + "|" for y in range(self.height)]
        rows.reverse()
        rows.append(" " + " ".join(str(i) for i in range(self.width)))
        print("\n".join(rows))


class Connect4Env(_BitboardEnv):
    """connect4env.py:11-101 (7x6 is the instantiated size)."""

    GAME = _lib.CONNECT4
    DEFAULT_WIDTH = 7
    DEFAULT_HEIGHT = 6

    def __init__(self, width=DEFAULT_WIDTH, height=DEFAULT_HEIGHT, state=None):
        super().__init__(width, height, width)
        if state is not None:
            self.set_state(state)

    @property
    def heights(self):
        return np.sum(np.abs(self.board), axis=1)

    def _info(self):
        return self.heights

    def get_state(self):
        return self.board, self.heights

    def variant_string(self):
        if (self.width, self.height) == (self.DEFAULT_WIDTH, self.DEFAULT_HEIGHT):
            return "connect4"
        return f"connect4_{self.width}_{self.height}"


class TicTacToeEnv(_BitboardEnv):
    """tictactoe_env.py:8-99 (3x3, three in a row)."""

    GAME = _lib.TICTACTOE
    DEFAULT_WIDTH = 3
    DEFAULT_HEIGHT = 3
    DEFAULT_WIN_AMOUNT = 3

    def __init__(self, width=DEFAULT_WIDTH, height=DEFAULT_HEIGHT, win_amount=DEFAULT_WIN_AMOUNT):
        super().__init__(width, height, width * height)
        self.win_amount = win_amount

    def get_loc(self, action):
        return np.unravel_index(action, (self.width, self.height))

    def variant_string(self):
        if (self.width, self.height, self.win_amount) == (3, 3, 3):
            return "tictactoe"
        return f"tictactoe_{self.width}_{self.height}_{self.win_amount}"
