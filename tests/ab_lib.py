"""The A/B library (make -C self_play_reinforcement_learning_amd/csrc ab: libspmcts_ab.so, -DSPMCTS_AB) holds
the measured-slower alternates and timing ablations behind environment switches; the product library refuses
those switches (SPMCTS_ERR_AB_SWITCH).  GPU tests of an alternate run it in a child process on this library."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(REPO, "self_play_reinforcement_learning_amd", "libspmcts_ab.so")


def ab_env(**switches):
    """Environment of a child process on the A/B library with the given switches set."""
    if not os.path.exists(AB_LIB):
        pytest.skip("A/B library not built (make -C self_play_reinforcement_learning_amd/csrc ab)")
    env = {k: v for k, v in os.environ.items() if k != "SPMCTS_LIB"}
    env["SPMCTS_LIB"] = AB_LIB
    env.update({k: str(v) for k, v in switches.items()})
    return env


def product_env():
    """Environment of a child process on the product library (no A/B switch set)."""
    env = {k: v for k, v in os.environ.items() if k != "SPMCTS_LIB" and not k.startswith(("SPMCTS_TOWER_", "SPMCTS_HEADS",
                                                                                            "SPMCTS_WIDE_", "SPMCTS_TREE_BLOCK",
                                                                                            "SPMCTS_EXPAND_CO", "SPMCTS_TREE_COPIES",
                                                                                            "SPMCTS_PEER_PUSH"))}
    return env


def run_child(code, env, *args, timeout=300):
    """Run `python -c code args...` from the repo root; returns its stdout (raises on a non-zero exit)."""
    r = subprocess.run([sys.executable, "-c", code, REPO, *map(str, args)], env=env, capture_output=True, text=True,
                       timeout=timeout, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout
