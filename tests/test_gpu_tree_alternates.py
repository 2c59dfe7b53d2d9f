"""GPU: the A/B library's alternates of the threaded tree kernels play the same games as the product kernels.

The alternates are kept for same-box A/B timing ("Steady-state tree phase"); a kept alternate that
drifted from the product's semantics would make those A/Bs meaningless, so each is held to bit-identical games:
scripts/rng_equal.py plays Connect4 and TicTacToe self-play games in Philox RNG mode with sequential (K = 1) and
threaded (K = 4) search on a ResNet, and every Move array and counter must match.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.ab_lib import REPO, ab_env, product_env

pytestmark = pytest.mark.gpu


def _games(env, out):
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "rng_equal.py"), str(out)], env=env, check=True,
                   timeout=600, cwd=REPO)
    return np.load(out)


@pytest.mark.parametrize("switches", [{"SPMCTS_TREE_COPIES": "1"}, {"SPMCTS_TREE_BLOCK": "8"}],
                         ids=["lds_block_copies", "one_tree_per_wave"])
def test_tree_alternates_play_identical_games(tmp_path, switches):
    ref = _games(product_env(), tmp_path / "product.npz")
    alt = _games(ab_env(**switches), tmp_path / "alt.npz")
    assert sorted(ref.files) == sorted(alt.files)
    for k in ref.files:
        assert np.array_equal(ref[k], alt[k]), k
