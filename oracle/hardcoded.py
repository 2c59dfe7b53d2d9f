"""Oracle restatement of the hard-coded players (games/general/hardcoded_players.py).
TEST INFRASTRUCTURE (see oracle/__init__.py).

Both keep their own env in their OWN frame: SelfPlayer.play_move passes
`player * -1` to the opposing policy (selfplayworker.py:221-224), so the
player's own stones are +1 there.  `player` is what reset(player) received
(selfplayworker.py:176: 1 if swap_sides else -1).

OneStepLookahead.__call__ (:18-33): among the valid moves, the first `a` for
which stepping a copy of the board with `step(a, self.player)` ends the game
(a win or a full board), else the first for which `step(a, -self.player)` does,
else `random.choice(valid moves)`.  Random.__call__ (:45-49): `random.choice`.

RNG: `rng.choice_index(n)` = the index random.choice picks among n moves.
PyRandomRNG reproduces the reference's global `random` stream (random.seed(s)
then random.choice(seq) = seq[_randbelow(len(seq))]); TapeRNG / RecordingRNG
(oracle/mcts.py) carry the same choice as one double (k + 0.5) / n, the form the
HIP arena's hard-coded players consume in tape mode (floor(u * n)).
"""
import random

from .envs import make_env


class PyRandomRNG:
    def __init__(self, seed):
        self.r = random.Random(seed)

    def choice_index(self, n):
        return self.r.choice(range(n))


class HardcodedPlayer:
    def __init__(self, kind, game, rng):
        if kind not in ("lookahead", "random"):
            raise ValueError(kind)
        self.kind = kind
        self.game = game
        self.rng = rng
        self.env = make_env(game)
        self.player = -1

    def reset(self, player=None):  # :35-37 / :51-52
        self.player = player
        self.env.reset()

    def play_action(self, action, player):  # :39-40 / :54-55
        self.env.step(action, player)

    def move(self):
        moves = [i for i, ok in enumerate(self.env.valid_moves()) if ok]
        if self.kind == "lookahead":
            for who in (self.player, -self.player):
                for a in moves:
                    test = make_env(self.game)
                    test.set_state(self.env.board.copy())
                    _, _, done, _ = test.step(a, who)
                    if done:
                        return a
        return moves[self.rng.choice_index(len(moves))]
