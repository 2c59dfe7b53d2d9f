"""CPU: the oracle (numpy restatement) reproduces the reference's own outputs (golden fixtures)."""
import json
import os

import numpy as np
import pytest

from oracle.envs import Connect4Env, GameOver, TicTacToeEnv
from oracle.mcts import NumpyRNG, OracleTree, RecordingRNG, TapeRNG
from oracle.selfplay import play_episode
from oracle.table_net import TableNet
from tests.parity_helpers import A_OF, load_json

pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


def _kat(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, f"env_kat_{name}.npz")))


@pytest.mark.parametrize("name,Env", [("c4", Connect4Env), ("ttt", TicTacToeEnv)])
def test_env_kat(golden_dir, name, Env):
    k = _kat(golden_dir, name)
    for i in range(len(k["action"])):
        e = Env()
        e.set_state(k["before"][i].astype(np.int64))
        if k["status"][i] == 2:
            e.episode_over = True
        try:
            s, r, d, _ = e.step(int(k["action"][i]), int(k["player"][i]))
            st = 0
        except ValueError:
            st, s = 1, e.board
        except GameOver:
            st, s = 2, e.board
        assert st == k["status"][i], i
        assert np.array_equal(s, k["after"][i]), i
        if st == 0:
            assert r == k["reward"][i] and d == k["done"][i], i
            assert np.array_equal(e.valid_moves(), k["valid"][i]), i


def test_env_kat_covers_all_win_directions(golden_dir):
    """The C4 KAT holds wins along rows, columns and both diagonals, and full-board draws."""
    k = _kat(golden_dir, "c4")
    seen = set()
    for i in np.nonzero((k["reward"] == 1) & (k["status"] == 0))[0]:
        b, p = k["after"][i].astype(int) * k["player"][i], None
        for name, (dx, dy) in {"h": (1, 0), "v": (0, 1), "d1": (1, 1), "d2": (1, -1)}.items():
            for x in range(7):
                for y in range(6):
                    if all(0 <= x + j * dx < 7 and 0 <= y + j * dy < 6 and b[x + j * dx, y + j * dy] == 1
                           for j in range(4)):
                        seen.add(name)
    assert seen == {"h", "v", "d1", "d2"}
    draws = (k["done"] & (k["reward"] == 0) & (k["status"] == 0))
    assert draws.any()
    assert (k["status"] == 1).any() and (k["status"] == 2).any()


@pytest.mark.parametrize("idx", range(0, 182, 1))
def test_mcts_search_matches_reference(idx):
    c = load_json("mcts_search.json")[idx]
    net = TableNet(A_OF[c["game"]], c["salt"])
    np.random.seed(c["seed"])
    t = OracleTree(c["game"], net, NumpyRNG(), c["sims"], strong_play=c["strong_play"])
    for a in c["opening"]:
        t.play_action(a)
    assert t.root.player == c["root_player"]
    a = t.move()
    st = t.root_stats()
    rec = t.temp_memory[-1]
    assert a == c["action"]
    assert st["child_n"] == c["child_n"] and st["child_w"] == c["child_w"]
    assert st["root_n"] == c["root_n"] and st["root_w"] == c["root_w"]
    assert rec["state"].reshape(-1).tolist() == c["state"]
    assert rec["tree_probs"].astype(float).tolist() == c["tree_probs"]
    assert float(rec["q"]) == c["q"]
    assert net.calls == c["net_calls"]


def test_tape_replay_equals_numpy_stream():
    """Recording the numpy stream and replaying it as a tape gives the identical search."""
    c = load_json("mcts_search.json")[30]
    A = A_OF[c["game"]]
    np.random.seed(c["seed"])
    rec = RecordingRNG(NumpyRNG())
    t1 = OracleTree(c["game"], TableNet(A, c["salt"]), rec, c["sims"])
    for a in c["opening"]:
        t1.play_action(a)
    a1 = t1.move()
    t2 = OracleTree(c["game"], TableNet(A, c["salt"]), TapeRNG(rec.tape), c["sims"])
    for a in c["opening"]:
        t2.play_action(a)
    a2 = t2.move()
    assert a1 == a2 and t1.root_stats() == t2.root_stats()


@pytest.mark.parametrize("idx", range(48))
def test_selfplay_games_match_reference(idx):
    g = load_json("selfplay_games.json")[idx]
    A = A_OF[g["game"]]
    net_p = TableNet(A, g["salt_policy"])
    net_o = net_p if not g["evaluate"] else TableNet(A, g["salt_opponent"])
    np.random.seed(g["seed"])
    rng = NumpyRNG()
    r, moves, log, _ = play_episode(g["game"], net_p, net_o, rng, rng, g["sims"], swap_sides=g["swap_sides"],
                                    update=not g["evaluate"], evaluate=g["evaluate"])
    assert r == g["result"]
    assert len(log) == len(g["plies"])
    for L, P in zip(log, g["plies"]):
        for k in ("tree", "action", "child_n", "child_w", "root_n", "root_w", "tree_probs", "q"):
            assert L[k] == P[k], k
    assert len(moves) == len(g["moves"])
    for m, M in zip(moves, g["moves"]):
        assert m["state"].reshape(-1).tolist() == M["state"]
        assert float(m["actual_val"]) == M["actual_val"]
        assert m["tree_probs"].astype(float).tolist() == M["tree_probs"]
        assert float(m["q"]) == M["q"]


def _g5_run(g, rng_p=None, rng_o=None):
    from oracle.hardcoded import PyRandomRNG

    A = A_OF[g["game"]]
    net_p = TableNet(A, g["salt_policy"])
    net_o = TableNet(A, g["salt_opponent"])
    np.random.seed(g["seed"])
    rng = NumpyRNG()
    if g["opponent"] != "mcts":
        rng_o = rng_o or PyRandomRNG(g["seed"])  # random.seed(seed) in the generator
    pkw, okw = g.get("policy_kwargs") or {}, g.get("opponent_kwargs") or {}
    return play_episode(g["game"], net_p, net_o, rng_p or rng, rng_o or rng, g["sims"],
                        swap_sides=g["swap_sides"], update=False, evaluate=True, opponent=g["opponent"],
                        opponent_iterations=g["opponent_sims"] or None, alpha=pkw.get("alpha", 1),
                        strong_play=pkw.get("strong_play", False), opponent_alpha=okw.get("alpha", 1),
                        opponent_strong_play=okw.get("strong_play", False))


@pytest.mark.parametrize("idx", range(66))
def test_evaluation_games_match_reference(idx):
    """G5: policy vs a second network with its own iteration count (and, games 44-65, its own alpha /
    strong_play), or vs OneStepLookahead / Random."""
    g = load_json("arena_games.json")[idx]
    r, moves, log, (pol, opp, env) = _g5_run(g)
    assert r == g["result"] and moves == []
    assert g["results_queue"] == [dict(reward=r, swap_sides=g["swap_sides"])]
    searched = [L for L in log if "child_n" in L]
    assert len(searched) == len(g["plies"])
    for L, P in zip(searched, g["plies"]):
        for k in ("tree", "action", "child_n", "child_w", "root_n", "root_w"):
            assert L[k] == P[k], k
    assert env.board.reshape(-1).astype(int).tolist() == g["final_board"]
    if g["opponent"] != "mcts":  # the hard-coded player's random.choice draws, in order
        from oracle.hardcoded import PyRandomRNG

        class Log(PyRandomRNG):
            def __init__(self, seed):
                super().__init__(seed)
                self.log = []

            def choice_index(self, n):
                k = super().choice_index(n)
                self.log.append([n, k])
                return k

        lg = Log(g["seed"])
        _g5_run(g, rng_o=lg)
        assert lg.log == g["choices"]


# ----------------------------------------------------------------- threaded (virtual-loss) mode
def _threaded_tree(c, threads):
    net = TableNet(A_OF[c["game"]], c["salt"])
    np.random.seed(c["seed"])
    t = OracleTree(c["game"], net, NumpyRNG(), c["sims"], strong_play=c["strong_play"], threads=threads)
    for a in c["opening"]:
        t.play_action(a)
    return t


def _walk(node):
    yield node
    for ch in node.children:
        yield from _walk(ch)


@pytest.mark.parametrize("idx", range(0, 182, 7))
@pytest.mark.parametrize("threads", [2, 4, 8])
def test_threaded_search_invariants(idx, threads):
    """K sims in flight (mcts.py:328-331): every sim is backed up or leaks its path's virtual loss;
    no lock survives the search; visit counts add up."""
    c = load_json("mcts_search.json")[idx]
    t = _threaded_tree(c, threads)
    n0, s0 = t.root.n, dict(t.stats)
    k0 = sum(ch.n for ch in t.root.children)
    t.move()
    sims = t.stats["sims"] - s0["sims"]
    leaks = t.stats["leaks"] - s0["leaks"]
    assert sims + leaks == c["sims"]
    assert t.root.n - n0 == sims
    nodes = list(_walk(t.root))
    assert not any(x.locked for x in nodes)
    assert all(x.vl >= 0 for x in nodes)
    if leaks == 0:
        assert all(x.vl == 0 for x in nodes)
    else:
        assert t.root.vl == leaks
    assert sum(ch.n for ch in t.root.children) - k0 == sims  # each backed-up sim passes one root child


def test_threaded_k1_is_the_sequential_search():
    """threads=1 is the reference's sequential mode, pinned by the G2 fixtures."""
    for c in load_json("mcts_search.json")[:40:3]:
        a = _threaded_tree(c, 1)
        act = a.move()
        assert act == c["action"] and a.root_stats()["child_n"] == c["child_n"]


def test_threaded_mode_changes_the_search():
    """K > 1 spreads the in-flight sims over more children (virtual loss discourages re-selection)."""
    cases = [c for c in load_json("mcts_search.json") if c["game"] == "connect4" and c["sims"] >= 25][:10]
    differ = 0
    for c in cases:
        a, b = _threaded_tree(c, 1), _threaded_tree(c, 8)
        a.move()
        b.move()
        differ += a.root_stats()["child_n"] != b.root_stats()["child_n"]
    assert differ > 0


@pytest.mark.parametrize("idx", range(0, 12, 3))
def test_threaded_episode_completes(idx):
    """oracle play_episode with K=4 sims in flight: a finished game, one Move per searched ply."""
    from oracle.selfplay import play_episode
    from oracle.mcts import RecordingRNG

    g = load_json("selfplay_games.json")[idx]
    A = A_OF[g["game"]]
    np.random.seed(g["seed"])
    base = NumpyRNG()
    r, moves, log, (pol, opp, env) = play_episode(g["game"], TableNet(A, g["salt_policy"]), TableNet(A, g["salt_policy"]),
                                                  RecordingRNG(base), RecordingRNG(base), g["sims"],
                                                  swap_sides=g["swap_sides"], threads=4)
    assert r in (-1, 0, 1)
    assert len(moves) == sum(1 for e in log if e["q"] is not None)
    for t in (pol, opp):
        assert all(x.vl >= 0 and not x.locked for x in _walk(t.root))
