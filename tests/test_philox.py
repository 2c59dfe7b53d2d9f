"""csrc/philox.h (the search's per-lane Philox draws) against rocRAND's own engine, on the host.

The arena's select / expand kernels draw child jitter from the tree's rocRAND Philox stream; the
header computes those draws from the state's counter, key and substate instead of rocRAND's
run-time-indexed output block (which forced the state through scratch memory).  This compiles
tests/philox_check.cpp with hipcc (host code only runs; no GPU) and requires bit-identical draws
and states.
"""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_philox_direct_draws_match_rocrand():
    src = os.path.join(ROOT, "tests", "philox_check.cpp")
    inc = os.path.join(ROOT, "self_play_reinforcement_learning_amd", "csrc")
    d = tempfile.mkdtemp()
    try:
        exe = os.path.join(d, "philox_check")
        subprocess.run([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950", "-I", inc, src, "-o", exe],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "mismatches 0" in r.stdout
    finally:
        shutil.rmtree(d, ignore_errors=True)
