"""MI355X-native batched self-play MCTS (drop-in for reubenvanammers/self_play_reinforcement_learning's
games/algos/mcts.py + games/algos/self_play_parallel.py hot path).

Public API mirrors the reference:
    MCTreeSearch, Move                    (games/algos/mcts.py)
    SelfPlayScheduler                     (games/algos/self_play_parallel.py)
    Memory                                (rl_utils/memory.py)
    ModelContainer, BasePlayer, Policy    (games/general/base_model.py)
    ResidualTower                         (games/general/modules.py)
    Connect4Env, TicTacToeEnv             (games/connect4, games/tictactoe)
    OneStepLookahead, Random              (games/general/hardcoded_players.py)
plus the arena itself: Arena, SelfPlayEngine, LanedEngine, DeviceTableNet.
"""
from .base_model import BasePlayer, ModelContainer, Policy, TrainableModel  # noqa: F401
from .memory import Memory  # noqa: F401
from .modules import InferenceTower, ResidualTower  # noqa: F401

_LAZY = {
    "Arena": ".arena",
    "SelfPlayEngine": ".engine",
    "LanedEngine": ".engine",
    "DeviceTableNet": ".evaluator",
    "make_evaluator": ".evaluator",
    "MCTreeSearch": ".mcts",
    "Move": ".mcts",
    "SelfPlayScheduler": ".self_play_parallel",
    "Connect4Env": ".envs",
    "TicTacToeEnv": ".envs",
    "GameOver": ".envs",
    "OneStepLookahead": ".hardcoded_players",
    "Random": ".hardcoded_players",
}


def __getattr__(name):
    if name in _LAZY:
        import importlib

        mod = importlib.import_module(_LAZY[name], __name__)
        return getattr(mod, name)
    raise AttributeError(name)
