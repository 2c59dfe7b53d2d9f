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
     as (n, index).  Later rows give the two MCTreeSearch sides their own
     alpha / strong_play (each side is built from its own container's kwargs,
     selfplayworker.py:71-81, mcts.py:119-136).

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
    plan = [  # game, EnvCls, A, policy sims, opponent kind, opponent sims, count[, policy kw, opponent kw]
        ("connect4", Connect4Env, 7, 25, "mcts", 40, 8),
        ("tictactoe", TicTacToeEnv, 9, 25, "mcts", 10, 8),
        ("connect4", Connect4Env, 7, 25, "lookahead", 0, 8),
        ("connect4", Connect4Env, 7, 25, "random", 0, 6),
        ("tictactoe", TicTacToeEnv, 9, 25, "lookahead", 0, 8),
        ("tictactoe", TicTacToeEnv, 9, 25, "random", 0, 6),
        # per-side search settings (round 3): the two sides differ in alpha and strong_play
        ("connect4", Connect4Env, 7, 25, "mcts", 30, 8, dict(alpha=1), dict(alpha=0.3, strong_play=True)),
        ("tictactoe", TicTacToeEnv, 9, 25, "mcts", 15, 8, dict(alpha=0.15, strong_play=True), dict(alpha=1)),
        ("connect4", Connect4Env, 7, 20, "mcts", 20, 6, dict(strong_play=True), dict(alpha=2.0)),
    ]
    games = []
    gid = 0
    try:
        for game, EnvCls, A, sims, kind, opp_sims, count, *kws in plan:
            pkw, okw = (kws + [{}, {}])[:2]
            for k in range(count):
                seed = 50_000 + gid
                swap = bool(k % 2)
                salt_p, salt_o = 5 * gid + 1, 5 * gid + 2
                np.random.seed(seed)
                random.seed(seed)
                rq = _ListQueue()
                pol = MCTreeSearch(network=TableNet(A, salt=salt_p), env=EnvCls, memory_queue=None, iterations=sims,
                                   **pkw)
                pol.train(False)
                if kind == "mcts":
                    opp = MCTreeSearch(network=TableNet(A, salt=salt_o), env=EnvCls, memory_queue=None,
                                       iterations=opp_sims, **okw)
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
                    policy_kwargs=pkw, opponent_kwargs=okw,
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


# ----------------------------------------------------------------------------- G7
def _record_pool(n, n_boards, seed):
    """n records over n_boards distinct Connect4 boards (so states repeat): int64 [7, 6] state,
    float32 scalar actual_val in {-1, 0, 1}, float32 [7] tree_probs, float32 scalar q."""
    rng = np.random.RandomState(seed)
    boards = []
    for _ in range(n_boards):
        b = np.zeros((7, 6), np.int64)
        h = [0] * 7
        p = 1
        for _ in range(rng.randint(0, 12)):
            c = rng.randint(7)
            if h[c] < 6:
                b[c, h[c]] = p
                h[c] += 1
                p = -p
        boards.append(b)
    pool = []
    for i in range(n):
        pool.append(dict(state=boards[rng.randint(n_boards)].reshape(-1).tolist(),
                         actual_val=float(rng.choice([-1.0, 0.0, 1.0])),
                         tree_probs=rng.dirichlet([0.7] * 7).astype(np.float32).astype(float).tolist(),
                         q=float(np.float32(rng.uniform(-1, 1)))))
    return pool


def gen_memory_ops():
    """The reference's Memory / Deduplicator (rl_utils/memory.py:8-94) driven through a fixed
    script of operations; every observable result is logged.  Records carry an `id` so that
    eviction / sampling / ordering can be logged; the key and value fields are tensors exactly as
    the reference's Move records (mcts.py:282-288, :230)."""
    from collections import namedtuple

    from games.algos.mcts import Move
    from rl_utils.memory import Memory

    Rec = namedtuple("Rec", ("state", "actual_val", "tree_probs"))
    pool = _record_pool(160, 14, seed=7)

    def rec(i, cls=Rec):
        d = pool[i]
        f = dict(state=torch.tensor(d["state"], dtype=torch.int64).view(7, 6),
                 actual_val=torch.tensor(d["actual_val"]).float(),
                 tree_probs=torch.tensor(d["tree_probs"], dtype=torch.float32))
        if cls is Move:
            f["q"] = torch.tensor(d["q"], dtype=torch.float32)
        r = cls(**f)
        return r

    def dump(buf):
        return [dict(state=r.state.reshape(-1).tolist(), actual_val=float(r.actual_val),
                     tree_probs=[float(x) for x in r.tree_probs.reshape(-1)]) for r in buf]

    ids = {}

    def add(mem, i, cls=Rec):
        r = rec(i, cls)
        ids[id(r)] = i
        mem.add(r)

    log = {}
    # 1. bounded ring, eviction, sampling, change_size
    m = Memory(50)
    for i in range(80):
        add(m, i)
    log["ring_after_80"] = [ids[id(r)] for r in m._buffer]
    np.random.seed(5)
    log["sample_seed5_k10"] = [ids[id(r)] for r in m.sample(10)]
    m.change_size(30)
    log["after_change_size_30"] = [ids[id(r)] for r in m._buffer]
    log["max_size_after_change"] = m.max_size
    # 2. deduplicate twice (persistent group table, maxlen rebinding the bound)
    m.deduplicate("state", ["actual_val", "tree_probs"], Rec)
    log["dedup1"] = dump(m._buffer)
    log["max_size_after_dedup1"] = m.max_size
    for i in range(80, 140):
        add(m, i)
    log["len_after_60_more"] = len(m)
    m.deduplicate("state", ["actual_val", "tree_probs"], Rec, maxlen=9)
    log["dedup2_maxlen9"] = dump(m._buffer)
    for i in range(140, 150):
        add(m, i)
    log["len_after_10_more"] = len(m)
    # 3. one-shot dedup of an unbounded memory (the comparison case for DeviceReplay)
    m2 = Memory()
    for i in range(120):
        add(m2, i)
    m2.deduplicate("state", ["actual_val", "tree_probs"], Rec)
    log["oneshot_120"] = dump(m2._buffer)
    # 4. get_duplicates
    m3 = Memory(100)
    for i in range(30):
        add(m3, i)
    groups, uniq = m3.get_duplicates("state")
    log["get_duplicates_groups"] = [[int(k), list(v)] for k, v in groups.items()]
    log["get_duplicates_unique"] = uniq.reshape(len(uniq), -1).tolist()
    # 5. the reference's own Move through deduplicate (mcts.py:385-386): the rebuilt tuple lacks q
    m4 = Memory(100)
    for i in range(40):
        add(m4, i, Move)
    try:
        m4.deduplicate("state", ["actual_val", "tree_probs"], Move)
        log["move_dedup_error"] = None
    except Exception as e:  # noqa: BLE001
        log["move_dedup_error"] = type(e).__name__
    log["move_dedup_buffer_after"] = dump(m4._buffer)
    log["move_dedup_len_after"] = len(m4)
    # 6. reset keeps max_size, empties
    m.reset()
    log["len_after_reset"] = len(m)
    return dict(pool=pool, log=log)


# ----------------------------------------------------------------------------- G8
def gen_trainer_step(ref_mcts, Connect4Env, ResidualTower):
    """The reference's training step: MCTreeSearch.update_from_memory (mcts.py:254-270) =
    Memory.sample (np.random.choice, rl_utils/memory.py:26-30) -> MCTreeSearch.loss (mcts.py:234-252,
    q_average adds the root q) -> SGD(lr, momentum 0.9, weight_decay 1e-4, self_play_parallel.py:193)
    step, two steps in a row (momentum), on seeded ResidualTower nets.  Modes: "train" (the
    UpdateWorker's policy.train(), updateworker.py:63: dropout + batch-stat BN, torch seeded per
    step), "train_nodrop" (the same with both dropout p set to 0: BN batch statistics without the
    CPU dropout stream, the form a GPU run can reproduce), "eval"."""
    from rl_utils.memory import Memory

    Move = ref_mcts.Move
    pool = _record_pool(96, 96, seed=11)
    out = {}
    batch_size, lr = 32, 0.01
    for name, kw, full in (("c4_tiny", dict(num_blocks=1, filter_factor=4), True),
                           ("c4_128x2", dict(num_blocks=2, filter_factor=32), False)):
        for mode in ("train", "train_nodrop", "eval"):
            torch.manual_seed(0)
            net = ResidualTower(width=7, height=6, action_size=7, **kw)
            net.eval()
            init = {k: v.detach().clone() for k, v in net.state_dict().items()}
            optim = torch.optim.SGD(net.parameters(), lr=lr, momentum=0.9, weight_decay=0.0001)
            pol = ref_mcts.MCTreeSearch(network=net, env=Connect4Env, optim=optim, batch_size=batch_size,
                                        memory_size=1000, min_memory=10)
            pol.memory = Memory(1000)
            recs = []
            for d in pool:
                r = Move(torch.tensor(d["state"], dtype=torch.int64).view(7, 6), torch.tensor(d["actual_val"]).float(),
                         torch.tensor(d["tree_probs"], dtype=torch.float32), torch.tensor(d["q"], dtype=torch.float32))
                recs.append(r)
                pol.memory.add(r)
            pol.train(mode != "eval")
            if mode == "train_nodrop":
                net.policy_dropout.p = 0.0
                net.value_dropout.p = 0.0
            losses, picks = [], []
            orig_loss, orig_sample = pol.loss, pol.memory.sample

            def spy_loss(batch):
                v = orig_loss(batch)
                losses.append(float(v))
                return v

            def spy_sample(k):
                b = orig_sample(k)
                picks.append([next(j for j, r in enumerate(recs) if r is x) for x in b])
                return b

            pol.loss, pol.memory.sample = spy_loss, spy_sample
            for step in range(2):
                np.random.seed(100 + step)
                torch.manual_seed(200 + step)
                pol.update_from_memory()
            key = f"{name}/{mode}"
            out[f"{key}/losses"] = np.array(losses, np.float64)
            out[f"{key}/picks"] = np.array(picks, np.int64)
            sd = net.state_dict()
            names = list(sd.keys())
            out[f"{key}/keys"] = np.array(names)
            for stat, fn in (("init_sum", lambda t: init[t].double().sum()),
                             ("sum", lambda t: sd[t].double().sum()),
                             ("delta_sum", lambda t: (sd[t].double() - init[t].double()).sum()),
                             ("delta_l2", lambda t: (sd[t].double() - init[t].double()).norm())):
                out[f"{key}/{stat}"] = np.array([float(fn(t)) for t in names], np.float64)
            for t in names:
                flat = sd[t].reshape(-1)
                if full:
                    out[f"{key}/sd/{t}"] = sd[t].numpy()
                elif flat.numel() and flat.dtype.is_floating_point:
                    idx = np.unique(np.linspace(0, flat.numel() - 1, 24).astype(np.int64))
                    out[f"{key}/pick_idx/{t}"] = idx
                    out[f"{key}/pick_val/{t}"] = flat[torch.from_numpy(idx)].numpy()
    out["pool/state"] = np.array([d["state"] for d in pool], np.int8)
    out["pool/actual_val"] = np.array([d["actual_val"] for d in pool], np.float32)
    out["pool/tree_probs"] = np.array([d["tree_probs"] for d in pool], np.float32)
    out["pool/q"] = np.array([d["q"] for d in pool], np.float32)
    out["config"] = np.array([batch_size, lr], np.float64)
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
    if only == ["G7"]:
        print("G7 memory ops ...", flush=True)
        with open(os.path.join(HERE, "memory_ops.json"), "w") as f:
            json.dump(gen_memory_ops(), f)
        return
    if only == ["G8"]:
        print("G8 trainer step ...", flush=True)
        np.savez_compressed(os.path.join(HERE, "trainer_step.npz"), **gen_trainer_step(ref_mcts, Connect4Env,
                                                                                       ResidualTower))
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
    print("G7 memory ops ...", flush=True)
    with open(os.path.join(HERE, "memory_ops.json"), "w") as f:
        json.dump(gen_memory_ops(), f)
    print("G8 trainer step ...", flush=True)
    np.savez_compressed(os.path.join(HERE, "trainer_step.npz"), **gen_trainer_step(ref_mcts, Connect4Env,
                                                                                   ResidualTower))
    print("(G6 threaded-search statistics: tests/golden/make_threaded_stats.py)")
    print("done")


if __name__ == "__main__":
    main()
