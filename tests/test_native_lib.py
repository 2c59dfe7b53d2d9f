"""CPU: the C-ABI library loads, exports every symbol include/spmcts.h declares, and its
host-compiled bitboard rules (the same csrc/board.h the kernels use) pass the env KATs."""
import ctypes
import os
import re

import numpy as np
import pytest

from self_play_reinforcement_learning_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "spmcts.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(spmcts_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
    assert sorted(names) == _lib.HEADER_SYMBOLS
    assert L.spmcts_version() == 1


def test_config_struct_layout():
    # 14 x int32 + 3 x double + 2 x uint64 = 56 + 24 + 16
    assert ctypes.sizeof(_lib.Config) == 96
    # ..., error_flags, reserved, leaked_sims, compactions, nn_rows, cache_rows
    assert ctypes.sizeof(_lib.Counters) == 8 * 8 + 6 * 8 + 8 + 8 + 8 + 8 + 8 + 8


@pytest.mark.parametrize("name,game,W,H", [("c4", 0, 7, 6), ("ttt", 1, 3, 3)])
def test_host_bitboard_step_matches_reference_kat(golden_dir, name, game, W, H):
    k = dict(np.load(os.path.join(golden_dir, f"env_kat_{name}.npz")))
    L = _lib.lib()
    A = W if game == 0 else W * H
    r, d = ctypes.c_int32(), ctypes.c_int32()
    valid = np.zeros(A, dtype=np.uint8)
    for i in range(len(k["action"])):
        if k["status"][i] == 2:
            continue  # GameOver is the env object's flag, not a board rule
        b = np.ascontiguousarray(k["before"][i].astype(np.int8))
        st = L.spmcts_env_step_host(game, W, H, b.ctypes.data_as(ctypes.c_void_p), int(k["action"][i]),
                                    int(k["player"][i]), ctypes.byref(r), ctypes.byref(d))
        assert st == k["status"][i], i
        assert np.array_equal(b, k["after"][i]), i
        if st == 0:
            assert r.value == k["reward"][i] and bool(d.value) == bool(k["done"][i]), i
            L.spmcts_valid_moves_host(game, W, H, b.ctypes.data_as(ctypes.c_void_p),
                                      valid.ctypes.data_as(ctypes.c_void_p))
            assert np.array_equal(valid.astype(bool), k["valid"][i]), i


def test_env_facade_plays_a_game():
    from self_play_reinforcement_learning_amd.envs import Connect4Env, GameOver

    e = Connect4Env()
    e.reset()
    for a, p in [(0, 1), (1, -1), (0, 1), (1, -1), (0, 1), (1, -1)]:
        _, r, d, _ = e.step(a, p)
        assert r == 0 and not d
    _, r, d, heights = e.step(0, 1)
    assert r == 1 and d and heights[0] == 4
    with pytest.raises(GameOver):
        e.step(2, -1)


@pytest.mark.parametrize("game", ["connect4", "tictactoe"])
def test_host_hardcoded_players_match_oracle(game):
    """OneStepLookahead / Random (host API twins of the device players) vs the oracle restatement."""
    import random

    from oracle.envs import make_env
    from oracle.hardcoded import HardcodedPlayer, PyRandomRNG
    from self_play_reinforcement_learning_amd.envs import Connect4Env, TicTacToeEnv
    from self_play_reinforcement_learning_amd.hardcoded_players import OneStepLookahead, Random

    Env = Connect4Env if game == "connect4" else TicTacToeEnv
    rng = np.random.default_rng(3)
    for case in range(150):
        ref = make_env(game)
        ref.reset()
        plays, player = [], 1
        for _ in range(int(rng.integers(0, 12 if game == "connect4" else 6))):
            legal = np.flatnonzero(ref.valid_moves())
            a = int(rng.choice(legal))
            _, _, done, _ = ref.step(a, player)
            if done:
                break
            plays.append((a, player))
            player = -player
        if ref.episode_over if hasattr(ref, "episode_over") else False:
            continue
        for kind, Cls in (("lookahead", OneStepLookahead), ("random", Random)):
            look = 1 if case % 2 else -1
            host = Cls(env=Env)
            host.reset(look)
            orc = HardcodedPlayer(kind, game, PyRandomRNG(case))
            orc.reset(look)
            for a, p in plays:
                host.play_action(a, p)
                orc.play_action(a, p)
            random.seed(case)
            assert host(None) == orc.move(), (case, kind, plays)


def test_config_field_offsets_match_header(tmp_path):
    """ctypes mirror vs the C header (gcc offsetof), incl. search_threads (K sims in flight)."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = [f for f, _ in _lib.Config._fields_]
    src = tmp_path / "off.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "spmcts.h"\nint main(void){\n' +
                   "".join(f'printf("%zu\\n", offsetof(spmcts_config, {n}));\n' for n in names) +
                   'printf("%zu\\n", sizeof(spmcts_config));\nreturn 0;}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got[:-1] == [getattr(_lib.Config, n).offset for n in names]
    assert got[-1] == ctypes.sizeof(_lib.Config)


def _kernel_handles(path):
    """Mangled names of the kernel handle symbols the library defines (nm; the device stubs excluded)."""
    import shutil
    import subprocess

    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return sorted(line.split()[-1] for line in out.splitlines()
                  if line.split() and "__device_stub__" not in line and line.split()[-1].startswith("_ZN5tower"))


def test_product_library_holds_only_the_shipped_trunk_kernels():
    """The product build (make; no -DSPMCTS_AB) has one trunk kernel set per (board shape, channels,
    dtype): 8 k_tower_dyn (device-count path: 7x6 and 3x3, C = 128 and 256, bf16 and fp16; since round 5
    the 7x6 C = 256 set is the 6-board one-buffer 16x16x32 tiles alone, tails included) and 8 k_tower
    (host-count path tiles, one per shape and dtype), every Cfg without a timing ablation (ABL = 0), the
    7x6 C = 128 trunk only as the 16x16x32 (M16) two-buffer tiles and the 7x6 C = 256 trunk only as the M16
    one-buffer tiles (tower_wide16.h), the co-resident heads only, and no ring / LDS-heads / ablation kernel."""
    path = _lib.LIB_PATH
    if os.path.basename(path) != "libspmcts.so":
        pytest.skip("SPMCTS_LIB points at another build")
    names = _kernel_handles(path)
    dyn = [n for n in names if n.startswith("_ZN5tower11k_tower_dyn")]
    host = [n for n in names if n.startswith("_ZN5tower7k_tower")]
    assert len(dyn) == 8 and len(host) == 8, (len(dyn), len(host))
    # the 7x6 C = 128 kernels: Cfg<128, 256, 7, 6, ..., M16 = true> only (mangled ...Lb0ELb1EE: ONEBUF, M16)
    c128 = [n for n in dyn + host if "CfgILi128ELi256ELi7ELi6E" in n]
    assert len(c128) == 4 and all("Lb0ELb1EE" in n for n in c128), c128
    assert not [n for n in dyn + host if "CfgILi128ELi192ELi7ELi6E" in n or "CfgILi128ELi128ELi7ELi6E" in n]
    # the 7x6 C = 256 kernels: Cfg<256, 256, 7, 6, ..., ONEBUF = true, M16 = true> only
    c256 = [n for n in dyn + host if "CfgILi256ELi" in n and "ELi7ELi6E" in n]
    assert len(c256) == 4 and all("CfgILi256ELi256ELi7ELi6E" in n and "Lb1ELb1EE" in n for n in c256), c256
    # Cfg<C, ROWS, W, H, CG, WAVES, ABL, ...>: the 7th argument is 0 in every instantiation
    cfgs = re.findall(r"(?:CfgI|NS1_I)Li(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", " ".join(dyn + host))
    assert cfgs and all(c[6] == "0" for c in cfgs)
    assert {(c[0], c[2], c[3]) for c in cfgs} == {("128", "7", "6"), ("256", "7", "6"), ("128", "3", "3"),
                                                 ("256", "3", "3")}
    assert not [n for n in names if "ring" in n or n.startswith("_ZN5tower7k_headsI")]
    assert len([n for n in names if n.startswith("_ZN5tower10k_heads_co")]) == 8


def test_product_library_refuses_ab_switches(monkeypatch):
    """An A/B-library switch in the environment is refused by the product library's tower entry
    points (SPMCTS_ERR_AB_SWITCH = -5) before anything is launched, instead of being ignored."""
    if os.path.basename(_lib.LIB_PATH) != "libspmcts.so":
        pytest.skip("SPMCTS_LIB points at another build")
    import subprocess
    import sys

    code = ("import ctypes, sys; sys.path.insert(0, %r); from self_play_reinforcement_learning_amd import _lib; "
            "L = _lib.lib(); print(L.spmcts_tower_forward(7, 6, 128, 20, None, 0, None, None, None, 0, None))" % REPO)
    env = dict(os.environ, SPMCTS_TOWER_CG="200")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.split()[-1] == "-5"
    env.pop("SPMCTS_TOWER_CG")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.split()[-1] == "0"  # batch 0: nothing to do, no GPU call
