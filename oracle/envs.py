"""Oracle restatement of the reference board environments (numpy).  TEST INFRASTRUCTURE.

Restates games/connect4/connect4env.py and games/tictactoe/tictactoe_env.py
(and the clone protocol of games/general/base_env.py:9-10).  Boards are
int64[W, H] indexed [column, row], row 0 = bottom, pieces +1 / -1.
"""
import numpy as np


class GameOver(Exception):
    """games/general/base_env.py:4-5"""


def _reward_through(board, x, y, player, need):
    """get_reward: connect4env.py:72-84 / tictactoe_env.py:63-75 (lines through (x, y))."""
    W = board.shape[0]
    horizontals = board[:, y]
    verticals = board[x, :]
    diagonal_1 = np.diagonal(board, offset=y - x)
    diagonal_2 = np.diagonal(np.flipud(board), offset=y - W + x + 1)
    for row in (horizontals, verticals, diagonal_1, diagonal_2):
        if _fold(row, player, need) == need:
            return 1
    return 0


def _fold(row, player, need):
    """reduce(_calc_win_in_a_row, row * player, 0): connect4env.py:80,86-92 / tictactoe_env.py:71,77-83.

    f(x, y) = need if x >= need; x + y if y > 0; else 0.  The fold ends at `need`
    iff the line holds a run of >= need consecutive `player` pieces.
    """
    x = 0
    for y in np.asarray(row) * player:
        if x >= need:
            x = need
            continue
        x = x + y if y > 0 else 0
    return need if x >= need else x


class Connect4Env:
    """connect4env.py:11-101"""

    def __init__(self, width=7, height=6):
        self.width, self.height = width, height
        self.n_actions = width
        self.reset()

    def max_moves(self):
        return self.width * self.height  # :25-26

    def reset(self):  # :50-54
        self.episode_over = False
        self.board = np.zeros([self.width, self.height], dtype=np.int64)
        self.heights = np.zeros([self.width], dtype=np.int64)
        return self.board

    def set_state(self, state):  # :56-58 (adopts by alias, heights = column |piece| sums)
        self.board = state
        self.heights = np.sum(np.abs(state), axis=1)

    def valid_moves(self):  # :47-48
        return self.heights < self.height

    def step(self, action, player=1):  # :29-43
        if self.episode_over:
            raise GameOver
        h = self.heights[action]
        if h < self.height:
            self.board[action, h] = player
            self.heights[action] += 1
        else:
            raise ValueError
        reward = _reward_through(self.board, action, self.heights[action] - 1, player, 4)
        self.episode_over = reward != 0 or int(np.sum(self.heights)) == self.height * self.width
        return self.board, reward, self.episode_over, self.heights

    def clone(self):  # base_env.py:9-10 (deepcopy)
        e = Connect4Env(self.width, self.height)
        e.board = self.board.copy()
        e.heights = self.heights.copy()
        e.episode_over = self.episode_over
        return e


class TicTacToeEnv:
    """tictactoe_env.py:8-99"""

    def __init__(self, width=3, height=3, win_amount=3):
        self.width, self.height, self.win_amount = width, height, win_amount
        self.n_actions = width * height
        self.reset()

    def max_moves(self):
        return self.width * self.height

    def reset(self):
        self.episode_over = False
        self.board = np.zeros([self.width, self.height], dtype=np.int64)
        return self.board

    def set_state(self, state):  # :36-37
        self.board = state

    def get_loc(self, action):  # :39-40  np.unravel_index(action, (W, H))
        return action // self.height, action % self.height

    def valid_moves(self):  # :42-43
        return self.board.reshape(-1) == 0

    def step(self, action, player=1):  # :23-33 (occupied cell = silent no-op)
        if self.episode_over:
            raise GameOver
        x, y = self.get_loc(action)
        if not self.board[x, y]:
            self.board[x, y] = player
        reward = _reward_through(self.board, x, y, player, self.win_amount)
        self.episode_over = reward != 0 or bool(self.board.all())
        return self.board, reward, self.episode_over, None

    def clone(self):
        e = TicTacToeEnv(self.width, self.height, self.win_amount)
        e.board = self.board.copy()
        e.episode_over = self.episode_over
        return e


def make_env(game):
    return {"connect4": Connect4Env, "tictactoe": TicTacToeEnv}[game]()
