"""Oracle restatement of one self-play episode (games/algos/selfplayworker.py:164-224).

TEST INFRASTRUCTURE (see oracle/__init__.py).  Two independent trees per game
(policy = tree 0, opposing = tree 1), each in its own frame (+1 = the tree's
owner, selfplayworker.py:175-176, :215-223); both trees advance on every ply
(play_move :221-224); the game env is in the policy's frame.
"""
import numpy as np

from .envs import make_env
from .hardcoded import HardcodedPlayer
from .mcts import OracleTree


def play_episode(game, net_policy, net_opponent, rng_policy, rng_opponent, iterations, swap_sides=False,
                 update=True, evaluate=False, alpha=1, strong_play=False, on_ply=None, opponent="mcts",
                 opponent_iterations=None, threads=1, opponent_alpha=None, opponent_strong_play=None,
                 opponent_threads=None):
    """SelfPlayer.play_episode (selfplayworker.py:172-194).

    The reference draws every random number from ONE global RandomState, in
    call order; pass the same NumpyRNG for both trees to reproduce it, or two
    TapeRNG streams (one per tree) to replay a recorded game.

    Evaluation games (set_up_policies(evaluate=True), selfplayworker.py:68-81): the
    opposing side may be a second network with its own `opponent_iterations`, or
    opponent="lookahead" / "random" (oracle/hardcoded.py, drawing from rng_opponent).

    Returns (result r in the policy's frame, moves pushed to the memory queue in
    push order [policy's then opponent's], per-ply log).

    threads=K > 1: both trees search with K sims in flight (oracle/mcts.py threaded mode).
    opponent_alpha / opponent_strong_play / opponent_threads: the opposing MCTreeSearch's own kwargs
    (selfplayworker.py:71-81 builds it from its own container); None = the policy's.
    """
    env = make_env(game)
    env.reset()
    pol = OracleTree(game, net_policy, rng_policy, iterations, alpha, strong_play, evaluate=evaluate,
                     root_player=(-1 if swap_sides else 1), threads=threads)
    if opponent == "mcts":
        opp = OracleTree(game, net_opponent, rng_opponent,
                         iterations if opponent_iterations is None else opponent_iterations,
                         alpha if opponent_alpha is None else opponent_alpha,
                         strong_play if opponent_strong_play is None else opponent_strong_play,
                         evaluate=evaluate, root_player=(1 if swap_sides else -1),
                         threads=threads if opponent_threads is None else opponent_threads)
    else:
        opp = HardcodedPlayer(opponent, game, rng_opponent)
        opp.reset(1 if swap_sides else -1)
    log = []

    def get_and_play(player):  # :209-219
        tree = pol if player == 1 else opp
        if isinstance(tree, HardcodedPlayer):
            a = tree.move()
            log.append(dict(tree=1, action=a))
            if on_ply is not None:
                on_ply(log[-1])
            pol.play_action(a)
            opp.play_action(a, -player)  # its own frame (play_move :221-224)
            _, r, done, _ = env.step(a, player=player)
            return r * player, done
        tree.search()
        stats = tree.root_stats()
        n_before = len(tree.temp_memory)
        a = tree._play(1)
        rec = tree.temp_memory[-1] if len(tree.temp_memory) > n_before else None
        log.append(dict(tree=0 if player == 1 else 1, action=a, **stats,
                        tree_probs=(rec["tree_probs"].astype(float).tolist() if rec is not None else None),
                        q=(float(rec["q"]) if rec is not None else None)))
        if on_ply is not None:
            on_ply(log[-1])
        # play_move (:221-224): both trees advance, then the env steps
        pol.play_action(a)
        if isinstance(opp, HardcodedPlayer):
            opp.play_action(a, -player)
        else:
            opp.play_action(a)
        _, r, done, _ = env.step(a, player=player)
        return r * player, done

    r = 0
    if swap_sides:
        get_and_play(-1)
    for _ in range(env.max_moves()):  # play_round (:196-203)
        r, done = get_and_play(1)
        if done:
            break
        r, done = get_and_play(-1)
        if done:
            break
    moves = []
    if update:
        moves += pol.push_result(r)
        if not isinstance(opp, HardcodedPlayer):
            moves += opp.push_result(-r)
    return int(r), moves, log, (pol, opp, env)
