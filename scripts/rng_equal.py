"""Same games from two library builds (Philox RNG mode, threaded and sequential search): run with
SPMCTS_LIB=<lib> and an output path, then `--compare a.npz b.npz`.  Used to check that a change of
how the per-lane draws are computed leaves every draw, and so every game, bit-identical."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def run(out):
    import torch

    from self_play_reinforcement_learning_amd.engine import SelfPlayEngine
    from self_play_reinforcement_learning_amd.modules import ResidualTower

    res = {}
    for game, W, H, A in (("connect4", 7, 6, 7), ("tictactoe", 3, 3, 9)):
        for threads in (1, 4):
            torch.manual_seed(0)
            net = ResidualTower(W, H, A, num_blocks=2, filter_factor=32)
            eng = SelfPlayEngine(game, net, n_games=256, iterations=24, seed=11, max_games=512,
                                 search_threads=threads)
            got = []
            eng.run(games=512, on_moves=lambda m: got.append({k: v.cpu().numpy() for k, v in m.items()}))
            eng.check()
            for k in got[0]:
                res[f"{game}_{threads}_{k}"] = np.concatenate([g[k] for g in got])
            c = eng.counters()
            res[f"{game}_{threads}_counters"] = np.array([c["sims"], c["nn_leaves"], c["depth_sum"], c["moves"]])
    np.savez(out, **res)


def compare(a, b):
    x, y = np.load(a), np.load(b)
    assert sorted(x.files) == sorted(y.files)
    bad = [k for k in x.files if not np.array_equal(x[k], y[k])]
    print("identical" if not bad else f"DIFFERENT: {bad}", len(x.files), "arrays")
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
