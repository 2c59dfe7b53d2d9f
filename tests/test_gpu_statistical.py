"""GPU, product RNG: root visit-count distributions of the Philox arena vs the reference's search.

The bit-exact parity tests drive the arena with the reference's own random stream (tape mode).
In product mode each tree draws from its own rocRAND Philox subsequence instead, so individual
searches differ from the reference's, but the DISTRIBUTION of search outcomes must not: here the
same position and deterministic table network are searched by N = 4,096 Philox trees on the GPU
and by M oracle searches driven by numpy's legacy RandomState exactly as the reference does
(oracle/mcts.py, pinned to the reference by G2/G3), and the mean root visit distribution (the
Move's tree_probs at temperature 1) and the chosen-action frequencies are compared.

Tolerance (stated): every component within 4.5 standard errors of the difference of the two
means (standard errors from the per-search sample variances of both sides) + 2e-3.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle_runs(game, sims, alpha, opening, salt, M):
    from oracle.mcts import NumpyRNG, OracleTree
    from oracle.table_net import TableNet

    A = 7 if game == "connect4" else 9
    net = TableNet(A, salt=salt)
    probs, acts = [], []
    for seed in range(M):
        np.random.seed(10_000 + seed)
        t = OracleTree(game, net, NumpyRNG(), sims, alpha=alpha)
        for a in opening:
            t.play_action(a)
        t.search()
        a = t._play(1)
        probs.append(np.asarray(t.temp_memory[-1]["tree_probs"], dtype=np.float64))
        acts.append(a)
    return np.stack(probs), np.asarray(acts)


def _gpu_runs(game, sims, alpha, opening, salt, N):
    from self_play_reinforcement_learning_amd.arena import Arena, table_net_eval
    from tests.parity_helpers import empty_prior

    arena = Arena(game, n_trees=N, iterations=sims, rng="philox", seed=123, alpha=alpha, leaf_format="f32")

    def step(count):
        if count:
            p, v = table_net_eval(game, arena.leaves(count), "f32", "nchw", salt=salt)
            arena.expand(p, v)

    arena.tree_reset(list(range(N)), [1] * N, priors=np.tile(empty_prior(game, salt), (N, 1)))
    for a in opening:
        step(arena.play_action(list(range(N)), [a] * N))
    arena.search_begin(list(range(N)))
    for _ in range(sims):
        step(arena.select())
    out = arena.search_end(1.0)
    arena.check()
    res = out["tree_probs"].double().cpu().numpy(), out["action"].cpu().numpy()
    arena.close()
    return res


@pytest.mark.parametrize("game,sims,alpha,opening,M", [
    ("connect4", 25, 1.0, [3, 3, 2], 2000),
    ("connect4", 60, 1.0, [], 1500),
    ("tictactoe", 25, 0.3, [4], 2000),
])
def test_philox_visit_distribution_matches_reference(game, sims, alpha, opening, M):
    salt, N = 4242, 4096
    cp, ca = _oracle_runs(game, sims, alpha, opening, salt, M)
    gp, ga = _gpu_runs(game, sims, alpha, opening, salt, N)
    A = cp.shape[1]
    np.testing.assert_allclose(gp.sum(1), 1.0, atol=1e-5)
    se = np.sqrt(cp.var(0, ddof=1) / M + gp.var(0, ddof=1) / N)
    diff = np.abs(cp.mean(0) - gp.mean(0))
    assert (diff <= 4.5 * se + 2e-3).all(), (cp.mean(0), gp.mean(0), se)
    fc = np.bincount(ca, minlength=A) / M
    fg = np.bincount(ga, minlength=A) / N
    sef = np.sqrt(fc * (1 - fc) / M + fg * (1 - fg) / N)
    assert (np.abs(fc - fg) <= 4.5 * sef + 2e-3).all(), (fc, fg)
    # the search is not degenerate: the noise spreads the visits over several actions
    assert (gp.mean(0) > 0.01).sum() >= 2


def test_statistical_check_has_power():
    """Negative control: the same comparison rejects a search whose root noise is drawn with a
    different Dirichlet alpha (so the tolerance above is not vacuous)."""
    game, sims, opening, salt, M, N = "tictactoe", 25, [4], 4242, 2000, 4096
    cp, _ = _oracle_runs(game, sims, 0.3, opening, salt, M)
    gp, _ = _gpu_runs(game, sims, 3.0, opening, salt, N)
    se = np.sqrt(cp.var(0, ddof=1) / M + gp.var(0, ddof=1) / N)
    diff = np.abs(cp.mean(0) - gp.mean(0))
    assert not (diff <= 4.5 * se + 2e-3).all()


def test_philox_visit_distribution_matches_reference_with_resnet():
    """Same comparison with a real ResidualTower (ResNet-128 trunk, 2 blocks): the oracle searches
    with the fp32 CPU network exactly as the reference does; the arena with the fused bf16 HIP tower
    and Philox.  bf16 leaf evaluation perturbs priors by ~1e-3, far below the sampling error."""
    from oracle.mcts import NumpyRNG, OracleTree
    from self_play_reinforcement_learning_amd.arena import Arena
    from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
    from self_play_reinforcement_learning_amd.modules import ResidualTower

    torch.manual_seed(3)
    net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=32).eval()
    sims, opening, M, N = 25, [3], 600, 4096
    torch.set_num_threads(8)
    cp, ca = [], []
    with torch.no_grad():
        for seed in range(M):
            np.random.seed(30_000 + seed)
            t = OracleTree("connect4", net, NumpyRNG(), sims)
            for a in opening:
                t.play_action(a)
            t.search()
            ca.append(t._play(1))
            cp.append(np.asarray(t.temp_memory[-1]["tree_probs"], dtype=np.float64))
    cp, ca = np.stack(cp), np.asarray(ca)

    ev = HipTowerEvaluator(net.cuda())
    arena = Arena("connect4", n_trees=N, iterations=sims, rng="philox", seed=99, leaf_format=ev.leaf_format,
                  leaf_layout=ev.leaf_layout)
    root_p, _ = ev(ev.empty_root_input(7, 6, arena.device))
    arena.set_root_prior(root_p[0])

    def step(count):
        if count:
            p, v = ev(arena.leaves(count))
            arena.expand(p, v)

    arena.tree_reset(list(range(N)), [1] * N)
    for a in opening:
        step(arena.play_action(list(range(N)), [a] * N))
    arena.search_begin(list(range(N)))
    for _ in range(sims):
        step(arena.select())
    out = arena.search_end(1.0)
    arena.check()
    gp, ga = out["tree_probs"].double().cpu().numpy(), out["action"].cpu().numpy()
    arena.close()
    se = np.sqrt(cp.var(0, ddof=1) / M + gp.var(0, ddof=1) / N)
    assert (np.abs(cp.mean(0) - gp.mean(0)) <= 4.5 * se + 2e-3).all(), (cp.mean(0), gp.mean(0), se)
    fc, fg = np.bincount(ca, minlength=7) / M, np.bincount(ga, minlength=7) / N
    sef = np.sqrt(fc * (1 - fc) / M + fg * (1 - fg) / N)
    assert (np.abs(fc - fg) <= 4.5 * sef + 2e-3).all(), (fc, fg)
