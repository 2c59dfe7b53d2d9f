"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden.py            # writes tests/golden/*.npz|json

The reference ships no tests, goldens or known-answer vectors, so
these fixtures are the only pin for the oracle and the HIP path.  The reference
is imported by path with five tiny stand-ins for its missing, non-arithmetic
dependencies (tests/golden/refshims: anytree.NodeMixin, gym.spaces.Discrete,
colorama, multiprocessing_logging).  Nothing of the reference is copied: only
inputs and the outputs it produced are written.

Fixtures
  G1 env_kat_c4.npz / env_kat_ttt.npz  env step known answers (Connect4Env.step
     connect4env.py:29-43, get_reward :72-92, valid_moves :47-48; TicTacToeEnv
     tictactoe_env.py:23-82), incl. GameOver / ValueError paths.
  G2 mcts_search.json  one MCTreeSearch move (mcts.py:177-367) after a random
     opening played through play_action/_set_node (mcts.py:188-209), driven by
     the deterministic TableNet, numpy legacy RNG seeded per case.
  G3 selfplay_games.json  full SelfPlayer.play_episode games
     (selfplayworker.py:172-224) with two trees, incl. the Move records pushed to
     the memory queue (mcts.py:225-232) and evaluate-mode games.
  G4 net_io.npz  ResidualTower (games/general/modules.py:43-125) forward outputs
     for seeded random-init nets, pinning the build's own net definition.
  G5 arena_games.json  evaluation games (SelfPlayWorker.set_up_policies(evaluate=True),
     selfplayworker.py:68-94; play_episode(update=False)): the policy MCTreeSearch
     against a second MCTreeSearch with its own table net and its own iteration
     count, or against the hard-coded OneStepLookahead / Random players
     (games/general/hardcoded_players.py), whose `random.choice` draws are logged
     as (n, index).

    python tests/golden/make_golden.py G5     # regenerate one fixture only
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, os.path.join(HERE, "refshims"))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import torch  # noqa: E402

from oracle.table_net import TableNet  # noqa: E402


def _ref_imports():
    os.chdir("/tmp")  # reference modules may write logs into cwd
    from games.algos import mcts as ref_mcts
    from games.algos.selfplayworker import SelfPlayer
    from games.connect4.connect4env import Connect4Env
    from games.general.base_env import GameOver
    from games.general.modules import ResidualTower
    from games.tictactoe.tictactoe_env import TicTacToeEnv

    return ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv, GameOver, ResidualTower


# ----------------------------------------------------------------------------- G5
class _ChoiceSpy:
    """Stands in for the `random` module inside hardcoded_players: forwards to the real
    global `random.choice` and logs (len(seq), index of the result)."""

    def __init__(self, log):
        self.log = log

    def choice(self, seq):
        x = random.choice(seq)
        self.log.append((len(seq), list(seq).index(x)))
        return x


def gen_arena_games(ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv):
    from games.general import hardcoded_players as hp

    MCTreeSearch = ref_mcts.MCTreeSearch
    orig_play = MCTreeSearch._play
    orig_random = hp.random
    log, choices = [], []

    def spy_play(self, temp=0.05):
        root = self.root_node
        pre = dict(tree=getattr(self, "_golden_tree", -1), child_n=[int(c.n) for c in root.children],
                   child_w=[float(c.w) for c in root.children], root_n=int(root.n), root_w=float(root.w))
        a = orig_play(self, temp)
        pre["action"] = int(a)
        log.append(pre)
        return a

    MCTreeSearch._play = spy_play
    hp.random = _ChoiceSpy(choices)
    plan = [  # game, EnvCls, A, policy sims, opponent kind, opponent sims, count
        ("connect4", Connect4Env, 7, 25, "mcts", 40, 8),
        ("tictactoe", TicTacToeEnv, 9, 25, "mcts", 10, 8),
        ("connect4", Connect4Env, 7, 25, "lookahead", 0, 8),
        ("connect4", Connect4Env, 7, 25, "random", 0, 6),
        ("tictactoe", TicTacToeEnv, 9, 25, "lookahead", 0, 8),
        ("tictactoe", TicTacToeEnv, 9, 25, "random", 0, 6),
    ]
    games = []
    gid = 0
    try:
        for game, EnvCls, A, sims, kind, opp_sims, count in plan:
            for k in range(count):
                seed = 50_000 + gid
                swap = bool(k % 2)
                salt_p, salt_o = 5 * gid + 1, 5 * gid + 2
                np.random.seed(seed)
                random.seed(seed)
                rq = _ListQueue()
                pol = MCTreeSearch(network=TableNet(A, salt=salt_p), env=EnvCls, memory_queue=None, iterations=sims)
                pol.train(False)
                if kind == "mcts":
                    opp = MCTreeSearch(network=TableNet(A, salt=salt_o), env=EnvCls, memory_queue=None,
                                       iterations=opp_sims)
                    opp._golden_tree = 1
                elif kind == "lookahead":
                    opp = hp.OneStepLookahead(env=EnvCls)
                else:
                    opp = hp.Random(env=EnvCls)
                opp.env = EnvCls()
                opp.train(False)
                pol.evaluate(True)  # set_up_policies(evaluate=True): both sides try their hardest
                opp.evaluate(True)
                pol._golden_tree = 0
                sp = SelfPlayer(pol, opp, EnvCls(), rq)
                del log[:]
                del choices[:]
                states, r = sp.play_episode(swap_sides=swap, update=False)
                games.append(dict(
                    id=gid, game=game, sims=sims, opponent=kind, opponent_sims=opp_sims, seed=seed,
                    swap_sides=swap, salt_policy=salt_p, salt_opponent=salt_o, result=int(r),
                    results_queue=[dict(reward=int(x["reward"]), swap_sides=bool(x["swap_sides"])) for x in rq.items],
                    plies=[dict(x) for x in log], choices=[list(c) for c in choices],
                    final_board=np.asarray(states[-1]).astype(int).reshape(-1).tolist(),
                ))
                gid += 1
    finally:
        MCTreeSearch._play = orig_play
        hp.random = orig_random
    return games


# ----------------------------------------------------------------------------- G1
def gen_env_kat_c4(Connect4Env, GameOver, n_games=1500, seed=1234):
    rng = random.Random(seed)
    before, after, action, player, reward, done, valid, status = [], [], [], [], [], [], [], []
    game_id, ply = [], []
    dirs = {"h": 0, "v": 0, "d1": 0, "d2": 0}
    for g in range(n_games):
        env = Connect4Env()
        env.reset()
        p = 1 if g % 2 == 0 else -1
        k = 0
        while True:
            legal = [i for i, m in enumerate(env.valid_moves()) if m]
            a = rng.choice(legal)
            b0 = env.board.copy()
            s, r, d, _ = env.step(a, p)
            before.append(b0.astype(np.int8))
            after.append(s.astype(np.int8))
            action.append(a)
            player.append(p)
            reward.append(r)
            done.append(bool(d))
            valid.append(env.valid_moves().astype(np.bool_))
            status.append(0)
            game_id.append(g)
            ply.append(k)
            k += 1
            if d:
                # a step after the game is over raises GameOver (connect4env.py:30-31)
                b1 = env.board.copy()
                try:
                    env.step(a, -p)
                    st = 0
                except GameOver:
                    st = 2
                except ValueError:
                    st = 1
                before.append(b1.astype(np.int8))
                after.append(env.board.copy().astype(np.int8))
                action.append(a)
                player.append(-p)
                reward.append(0)
                done.append(True)
                valid.append(env.valid_moves().astype(np.bool_))
                status.append(st)
                game_id.append(g)
                ply.append(k)
                break
            p = -p
        # full-column error path (connect4env.py:33-37) on a fresh env
        if g % 10 == 0:
            env2 = Connect4Env()
            env2.reset()
            col = rng.randrange(7)
            q = 1
            for _ in range(6):
                env2.step(col, q)  # alternating pieces: no vertical four
                q = -q
            b0 = env2.board.copy()
            try:
                env2.step(col, 1)
                st = 0
            except ValueError:
                st = 1
            before.append(b0.astype(np.int8))
            after.append(env2.board.copy().astype(np.int8))
            action.append(col)
            player.append(1)
            reward.append(0)
            done.append(False)
            valid.append(env2.valid_moves().astype(np.bool_))
            status.append(st)
            game_id.append(-1)
            ply.append(-1)
    return dict(
        before=np.stack(before), after=np.stack(after), action=np.array(action, np.int8),
        player=np.array(player, np.int8), reward=np.array(reward, np.int8), done=np.array(done),
        valid=np.stack(valid), status=np.array(status, np.int8), game_id=np.array(game_id, np.int32),
        ply=np.array(ply, np.int16),
    )


def gen_env_kat_ttt(TicTacToeEnv, GameOver):
    """Exhaustive: every position reachable by legal play, every action (legal or not) from it."""
    seen = {}
    stack = [(np.zeros((3, 3), np.int64), 1)]
    while stack:
        b, p = stack.pop()
        key = (b.tobytes(), p)
        if key in seen:
            continue
        seen[key] = (b.copy(), p)
        for a in range(9):
            env = TicTacToeEnv()
            env.reset()
            env.set_state(b.copy())
            if env.board[np.unravel_index(a, (3, 3))] != 0:
                continue
            s, r, d, _ = env.step(a, p)
            if not d:
                stack.append((s.copy(), -p))
    before, after, action, player, reward, done, valid, status = [], [], [], [], [], [], [], []
    for (bb, p) in seen.values():
        for a in range(9):
            env = TicTacToeEnv()
            env.reset()
            env.set_state(bb.copy())
            try:
                s, r, d, _ = env.step(a, p)
                st = 0
            except GameOver:
                s, r, d, st = env.board, 0, True, 2
            before.append(bb.astype(np.int8))
            after.append(np.asarray(s).astype(np.int8))
            action.append(a)
            player.append(p)
            reward.append(r)
            done.append(bool(d))
            valid.append(env.valid_moves().astype(np.bool_))
            status.append(st)
    return dict(
        before=np.stack(before), after=np.stack(after), action=np.array(action, np.int8),
        player=np.array(player, np.int8), reward=np.array(reward, np.int8), done=np.array(done),
        valid=np.stack(valid), status=np.array(status, np.int8),
    )


# ----------------------------------------------------------------------------- G2
def _random_opening(EnvCls, rng, max_len):
    env = EnvCls()
    env.reset()
    acts = []
    p = 1
    for _ in range(rng.randrange(max_len + 1)):
        legal = [i for i, m in enumerate(env.valid_moves()) if m]
        # keep the opening non-terminal
        ok = []
        for a in legal:
            e2 = EnvCls()
            e2.reset()
            e2.set_state(env.board.copy())
            _, _, d, _ = e2.step(a, p)
            if not d:
                ok.append(a)
        if not ok:
            break
        a = rng.choice(ok)
        env.step(a, p)
        acts.append(a)
        p = -p
    return acts


def gen_mcts_search(ref_mcts, Connect4Env, TicTacToeEnv):
    MCTreeSearch = ref_mcts.MCTreeSearch
    cases = []
    plan = [
        ("connect4", Connect4Env, 7, 25, 60, 10, False),
        ("connect4", Connect4Env, 7, 200, 24, 12, False),
        ("connect4", Connect4Env, 7, 800, 6, 12, False),
        ("connect4", Connect4Env, 7, 200, 8, 30, True),
        ("tictactoe", TicTacToeEnv, 9, 25, 60, 4, False),
        ("tictactoe", TicTacToeEnv, 9, 200, 16, 5, False),
        ("tictactoe", TicTacToeEnv, 9, 200, 8, 5, True),
    ]
    cid = 0
    for game, EnvCls, A, sims, count, max_open, strong in plan:
        for k in range(count):
            rng = random.Random(1000 * sims + k + (7 if strong else 0) + (0 if game == "connect4" else 50000))
            opening = _random_opening(EnvCls, rng, max_open)
            seed = 10_000 + cid
            salt = cid * 7919
            net = TableNet(A, salt=salt)
            np.random.seed(seed)
            tree = MCTreeSearch(network=net, env=EnvCls, iterations=sims, strong_play=strong)
            for a in opening:
                tree.play_action(a, None)
            root_player = int(tree.root_node.player)
            tree.train(False)
            tree.evaluate(False)
            action = tree()
            root = tree.root_node
            mv = tree.temp_memory[-1] if tree.temp_memory else None
            kids = root.children
            cases.append(
                dict(
                    id=cid, game=game, sims=sims, seed=seed, salt=salt, strong_play=strong,
                    opening=opening, root_player=root_player, action=int(action),
                    child_n=[int(c.n) for c in kids], child_w=[float(c.w) for c in kids],
                    root_n=int(root.n), root_w=float(root.w),
                    recorded=mv is not None,
                    state=(mv.state.numpy().astype(int).reshape(-1).tolist() if mv else None),
                    tree_probs=(mv.tree_probs.numpy().astype(float).tolist() if mv else None),
                    q=(float(mv.q) if mv else None),
                    net_calls=net.calls,
                )
            )
            cid += 1
    return cases


# ----------------------------------------------------------------------------- G3
class _ListQueue:
    def __init__(self):
        self.items = []

    def put(self, x):
        self.items.append(x)

    def empty(self):
        return not self.items


def gen_selfplay_games(ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv):
    MCTreeSearch = ref_mcts.MCTreeSearch
    orig_play = MCTreeSearch._play
    log = []

    def spy_play(self, temp=0.05):
        root = self.root_node
        pre = dict(
            tree=getattr(self, "_golden_tree", -1),
            child_n=[int(c.n) for c in root.children],
            child_w=[float(c.w) for c in root.children],
            root_n=int(root.n), root_w=float(root.w),
        )
        a = orig_play(self, temp)
        pre["action"] = int(a)
        mv = self.temp_memory[-1] if self.temp_memory else None
        pre["tree_probs"] = mv.tree_probs.numpy().astype(float).tolist() if mv else None
        pre["q"] = float(mv.q) if mv else None
        log.append(pre)
        return a

    MCTreeSearch._play = spy_play
    games = []
    plan = [
        ("connect4", Connect4Env, 7, 25, 16, False),
        ("connect4", Connect4Env, 7, 200, 4, False),
        ("tictactoe", TicTacToeEnv, 9, 25, 16, False),
        ("connect4", Connect4Env, 7, 25, 6, True),  # evaluate mode (temp/20, mcts.py:272-276)
        ("tictactoe", TicTacToeEnv, 9, 25, 6, True),
    ]
    gid = 0
    try:
        for game, EnvCls, A, sims, count, evaluate in plan:
            for k in range(count):
                seed = 20_000 + gid
                swap = bool(k % 2)
                salt_p = 3 * gid + 1
                salt_o = salt_p if not evaluate else 3 * gid + 2
                np.random.seed(seed)
                mq = _ListQueue()
                rq = _ListQueue()
                net_p = TableNet(A, salt=salt_p)
                net_o = net_p if not evaluate else TableNet(A, salt=salt_o)
                pol = MCTreeSearch(network=net_p, env=EnvCls, memory_queue=mq, iterations=sims)
                pol.train(False)
                opp = MCTreeSearch(network=net_o, env=EnvCls, memory_queue=mq, iterations=sims)
                opp.env = EnvCls()
                opp.train(False)
                pol.evaluate(evaluate)
                opp.evaluate(evaluate)
                pol._golden_tree = 0
                opp._golden_tree = 1
                sp = SelfPlayer(pol, opp, EnvCls(), rq)
                del log[:]
                _, r = sp.play_episode(swap_sides=swap, update=not evaluate)
                moves = [
                    dict(
                        state=m.state.numpy().astype(int).reshape(-1).tolist(),
                        actual_val=float(m.actual_val), tree_probs=m.tree_probs.numpy().astype(float).tolist(),
                        q=float(m.q),
                    )
                    for m in mq.items
                ]
                games.append(
                    dict(
                        id=gid, game=game, sims=sims, seed=seed, swap_sides=swap, evaluate=evaluate,
                        salt_policy=salt_p, salt_opponent=salt_o, result=int(r),
                        results_queue=[dict(reward=int(x["reward"]), swap_sides=bool(x["swap_sides"])) for x in rq.items],
                        plies=[dict(x) for x in log], moves=moves,
                    )
                )
                gid += 1
    finally:
        MCTreeSearch._play = orig_play
    return games


# ----------------------------------------------------------------------------- G4
def gen_net_io(ResidualTower, Connect4Env, TicTacToeEnv):
    out = {}
    rng = random.Random(77)

    def boards(EnvCls, n):
        bs, ps = [], []
        for _ in range(n):
            env = EnvCls()
            env.reset()
            p = 1
            for _ in range(rng.randrange(8)):
                legal = [i for i, m in enumerate(env.valid_moves()) if m]
                _, _, d, _ = env.step(rng.choice(legal), p)
                if d:
                    env.reset()
                p = -p
            bs.append(env.board.copy())
            ps.append(rng.choice([1, -1]))
        return np.stack(bs), np.array(ps)

    specs = [
        ("c4_tiny", Connect4Env, dict(width=7, height=6, action_size=7, num_blocks=1, filter_factor=4), True),
        ("ttt_tiny", TicTacToeEnv, dict(width=3, height=3, action_size=9, num_blocks=1, filter_factor=4), True),
        ("c4_128x2", Connect4Env, dict(width=7, height=6, action_size=7, num_blocks=2, filter_factor=32), False),
    ]
    for name, EnvCls, kw, store_weights in specs:
        torch.manual_seed(0)
        net = ResidualTower(**kw)
        net.eval()
        b, p = boards(EnvCls, 32)
        with torch.no_grad():
            probs, val = net.forward(torch.tensor(b * p[:, None, None]))
            single = [net(b[i], int(p[i])) for i in range(4)]
        out[f"{name}/boards"] = b.astype(np.int8)
        out[f"{name}/players"] = p.astype(np.int8)
        out[f"{name}/probs"] = probs.numpy().astype(np.float32)
        out[f"{name}/values"] = val.numpy().astype(np.float32).reshape(-1)
        out[f"{name}/single_probs"] = np.array([s[0] for s in single], np.float32)
        out[f"{name}/single_values"] = np.array([s[1] for s in single], np.float64)
        sd = net.state_dict()
        out[f"{name}/keys"] = np.array(list(sd.keys()))
        out[f"{name}/shapes"] = np.array([",".join(map(str, v.shape)) for v in sd.values()])
        out[f"{name}/checksums"] = np.array([float(v.double().sum()) for v in sd.values()], np.float64)
        if store_weights:
            for k, v in sd.items():
                out[f"{name}/sd/{k}"] = v.numpy()
    return out


def main():
    ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv, GameOver, ResidualTower = _ref_imports()
    torch.set_num_threads(4)
    only = sys.argv[1:]
    if only == ["G5"]:
        print("G5 arena games ...", flush=True)
        with open(os.path.join(HERE, "arena_games.json"), "w") as f:
            json.dump(gen_arena_games(ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv), f)
        return
    print("G1 env KATs ...", flush=True)
    np.savez_compressed(os.path.join(HERE, "env_kat_c4.npz"), **gen_env_kat_c4(Connect4Env, GameOver))
    np.savez_compressed(os.path.join(HERE, "env_kat_ttt.npz"), **gen_env_kat_ttt(TicTacToeEnv, GameOver))
    print("G2 MCTS searches ...", flush=True)
    cases = gen_mcts_search(ref_mcts, Connect4Env, TicTacToeEnv)
    with open(os.path.join(HERE, "mcts_search.json"), "w") as f:
        json.dump(cases, f)
    print("G3 self-play games ...", flush=True)
    games = gen_selfplay_games(ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv)
    with open(os.path.join(HERE, "selfplay_games.json"), "w") as f:
        json.dump(games, f)
    print("G4 net I/O ...", flush=True)
    np.savez_compressed(os.path.join(HERE, "net_io.npz"), **gen_net_io(ResidualTower, Connect4Env, TicTacToeEnv))
    print("G5 arena games ...", flush=True)
    with open(os.path.join(HERE, "arena_games.json"), "w") as f:
        json.dump(gen_arena_games(ref_mcts, SelfPlayer, Connect4Env, TicTacToeEnv), f)
    print("done")


if __name__ == "__main__":
    main()
