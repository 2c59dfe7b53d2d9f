"""Hard-coded opponents with the reference API (games/general/hardcoded_players.py:8-56).

`OneStepLookahead` and `Random` keep the reference's BasePlayer surface for
interactive play on the host envs (`__call__(s) -> action`, `reset(player)`,
`play_action(action, player)`).  Passed as the `policy_gen` of an
`evaluation_policy_container`, they make `SelfPlayScheduler.compare_models` /
evaluation games run them ON THE DEVICE as arena players
(`SPMCTS_PLAYER_LOOKAHEAD` / `SPMCTS_PLAYER_RANDOM`, csrc/spmcts.hip
`hardcoded_move`) against the policy's trees.
"""
import random

from .base_model import BasePlayer


class OneStepLookahead(BasePlayer):
    """Win if a move ends the game for `player`, else block one that ends it for `-player`,
    else a random valid move (hardcoded_players.py:18-33; `done` includes a full board)."""

    def __init__(self, env, player=-1, **kwargs):
        self.env = env()
        self.env_gen = env
        self.player = player

    def __call__(self, s):
        state = self.env.get_state()[0].copy()
        possible_moves = [i for i, ok in enumerate(self.env.valid_moves()) if ok]
        test_env = self.env_gen()
        for who in (self.player, -self.player):
            for a in possible_moves:
                test_env.set_state(state.copy())
                _, _, done, _ = test_env.step(a, who)
                if done:
                    return a
        return random.choice(possible_moves)

    def reset(self, player=None):
        self.player = player
        self.env.reset()

    def play_action(self, action, player):
        self.env.step(action, player)


class Random(BasePlayer):
    """A uniformly random valid move (hardcoded_players.py:36-56)."""

    def __init__(self, env, player=-1, **kwargs):
        self.env = env()
        self.env_gen = env
        self.player = player

    def __call__(self, s):
        return random.choice([i for i, ok in enumerate(self.env.valid_moves()) if ok])

    def reset(self, player=None):
        self.env.reset()

    def play_action(self, action, player):
        self.env.step(action, player)
