"""GPU: the fused HIP residual-tower kernel computes the reference network.

Numerics: bf16 or fp16 MFMA with fp32 accumulation and bf16 / fp16 activations between layers.
Tolerance: the fused kernel's deviation from the fp32 reference forward
(games/general/modules.py:88-107, eval mode) must be within 2x the deviation of
PyTorch's own path in the same dtype on the same inputs (+2e-3; for fp16 that path is
the reference's own inference mode, torch.autocast fp16, inference_worker.py:117), and
below 0.05 absolute on probabilities and values.  Each board is computed independently,
so a board's output is bit-identical whatever batch it is evaluated in.
"""
import numpy as np
import pytest
import torch

from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator, TowerEvaluator
from self_play_reinforcement_learning_amd.modules import ResidualTower, planes_from_boards

pytestmark = pytest.mark.gpu


def _net(W, H, A, blocks, ff, seed=0):
    torch.manual_seed(seed)
    net = ResidualTower(W, H, A, num_blocks=blocks, filter_factor=ff)
    with torch.no_grad():  # non-trivial eval statistics so BN folding is exercised
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.weight.uniform_(0.6, 1.4)
                m.bias.uniform_(-0.1, 0.1)
    return net.cuda().eval()


def _planes(W, H, n, seed=1):
    rng = np.random.default_rng(seed)
    b = rng.choice([-1, 0, 1], size=(n, W, H), p=[0.3, 0.4, 0.3])
    return planes_from_boards(torch.as_tensor(b), W, H).cuda()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("game,blocks,ff", [("connect4", 2, 32), ("connect4", 20, 32), ("connect4", 2, 64),
                                             ("connect4", 20, 64), ("tictactoe", 3, 32)])
def test_tower_matches_fp32_reference(game, blocks, ff, dtype):
    W, H, A = (7, 6, 7) if game == "connect4" else (3, 3, 9)
    net = _net(W, H, A, blocks, ff)
    x = _planes(W, H, 777)
    with torch.no_grad():
        ref_p, ref_v = net.forward_planes(x)
    hip = HipTowerEvaluator(net, dtype=dtype)
    xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    p, v = hip(xb)
    if dtype == torch.float16:  # the reference's inference: fp32 module under fp16 autocast
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            p2, v2 = net.forward_planes(x)
        p2, v2 = p2.float(), v2.float().view(-1)
    else:
        p2, v2 = TowerEvaluator(net, dtype=torch.bfloat16)(xb)
    for mode in (False, "gemm"):  # torch heads / GEMM + epilogue heads vs the default MFMA heads kernel
        p3, v3 = HipTowerEvaluator(net, fused_heads=mode, dtype=dtype)(xb)
        assert (p - p3).abs().max().item() < 1e-2 and (v - v3).abs().max().item() < 1e-2
    e_hip = max((p - ref_p).abs().max().item(), (v - ref_v.view(-1)).abs().max().item())
    e_bf = max((p2 - ref_p).abs().max().item(), (v2 - ref_v.view(-1)).abs().max().item())
    assert e_hip <= 2 * e_bf + 2e-3, (e_hip, e_bf)
    assert e_hip < 0.05
    torch.testing.assert_close(p.sum(1), torch.ones(p.shape[0], device=p.device), atol=1e-5, rtol=0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("ff", [32, 64])  # C = 128 (tower_m16.h) and C = 256 (tower_wide16.h)
def test_tower_rows_independent_of_batch(dtype, ff):
    net = _net(7, 6, 7, 2, ff)
    hip = HipTowerEvaluator(net, dtype=dtype)
    x = _planes(7, 6, 1000, seed=5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    full_p, full_v = hip(x)
    for n in (1, 4, 5, 6, 7, 13, 255, 1000):
        p, v = hip(x[:n])
        assert torch.equal(p, full_p[:n]) and torch.equal(v, full_v[:n]), n
    # offset windows: a board's result does not depend on its neighbours in the tile
    p, v = hip(x[3:40])
    assert torch.equal(p, full_p[3:40]) and torch.equal(v, full_v[3:40])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [1, 37, 700, 1536, 2336, 4000])
@pytest.mark.parametrize("ff", [32, 64])
def test_forward_dev_matches_host_count(n, dtype, ff):
    """The device-count launch (row count read on device, full/middle/half workgroups chosen on
    device) gives the host-count results bit for bit on the live rows.  On 256 CUs, 2,336 and 4,000
    rows leave tails of 800 and 928 boards: one round of the 4-board middle tile."""
    W, H, A = 7, 6, 7
    net = _net(W, H, A, 2, ff)
    max_rows = 4096
    x = _planes(W, H, max_rows, seed=5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    hip = HipTowerEvaluator(net, dtype=dtype)
    p, v = hip(x[:n].contiguous(memory_format=torch.channels_last))
    cnt = torch.tensor([n], dtype=torch.int32, device=x.device)
    for pack in (False, True):  # round-aligned tiles / SPMCTS_TOWER_PACK (full tiles + one small tail)
        hip.concurrent = pack
        pd, vd = hip.forward_dev(x, cnt, max_rows)
        torch.cuda.synchronize()
        assert torch.equal(pd[:n], p) and torch.equal(vd[:n].view(-1), v.view(-1)), pack


def test_engine_async_matches_sync_path():
    """A ply loop driven by the device-side leaf count reproduces the host-synchronised loop exactly."""
    from self_play_reinforcement_learning_amd.engine import SelfPlayEngine

    net = _net(7, 6, 7, 2, 32)
    out = []
    for async_device in (True, False):
        eng = SelfPlayEngine("connect4", net, n_games=48, iterations=12, seed=7, max_games=48)
        assert eng.evaluator.supports_device_count
        eng.async_device = async_device
        got = []
        eng.run(games=48, on_moves=lambda m: got.append({k: v.cpu().numpy() for k, v in m.items()}))
        eng.check()
        c = eng.counters()
        out.append(({k: np.concatenate([g[k] for g in got]) for k in got[0]}, c))
    (m1, c1), (m2, c2) = out
    for k in m1:
        np.testing.assert_array_equal(m1[k], m2[k], err_msg=k)
    for k in ("sims", "moves", "nn_leaves", "terminal_leaves", "depth_sum", "games_finished"):
        assert c1[k] == c2[k], k


def test_zero_and_maximum_rows():
    """Empty batches launch nothing and fail nothing; a device count above the buffer capacity is
    clamped inside the kernels (no write past the caller's buffers)."""
    net = _net(7, 6, 7, 2, 32)
    hip = HipTowerEvaluator(net)
    x = _planes(7, 6, 64, seed=9).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    p, v = hip(x[:0])
    assert p.shape[0] == 0 and v.shape[0] == 0
    cnt = torch.tensor([0], dtype=torch.int32, device=x.device)
    hip.forward_dev(x, cnt, 64)
    torch.cuda.synchronize()
    # count 10,000 into 64-row buffers guarded by 64 extra sentinel rows
    hip._dev_bufs = None
    hip.reserve(128, x.device)
    feats, probs, values = hip._dev_bufs
    probs.fill_(-7.0)
    values.fill_(-7.0)
    cnt.fill_(10_000)
    hip.forward_dev(x, cnt, 64)
    torch.cuda.synchronize()
    assert (probs[64:] == -7.0).all() and (values[64:] == -7.0).all()
    ref_p, ref_v = hip(x)
    assert torch.equal(probs[:64], ref_p) and torch.equal(values[:64].view(-1), ref_v.view(-1))


_HEADS_CASES = [("connect4", 1, 32), ("connect4", 31, 32), ("connect4", 33, 32), ("connect4", 1000, 32),
                ("connect4", 4096, 32), ("tictactoe", 77, 32), ("connect4", 33, 64), ("connect4", 1000, 64),
                ("tictactoe", 77, 64)]

_HEADS_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from tests.test_gpu_tower import _net, _planes, _HEADS_CASES
from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
out = {}
for dt, name in ((torch.bfloat16, "bf16"), (torch.float16, "fp16")):
    for game, n, ff in _HEADS_CASES:
        W, H, A = (7, 6, 7) if game == "connect4" else (3, 3, 9)
        x = _planes(W, H, n, seed=11).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        p, v = HipTowerEvaluator(_net(W, H, A, 2, ff), dtype=dt)(x)
        key = f"{name}_{game}_{n}_{ff}"
        out["p_" + key], out["v_" + key] = p.float().cpu().numpy(), v.float().cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def test_coresident_heads_match_lds_heads(tmp_path):
    """k_heads_co (the product library's heads: features read from global memory, 32 boards per workgroup,
    96 registers, so it fits beside a trunk workgroup; C = 256: two value passes) gives the LDS-staged k_heads'
    results (the A/B library's SPMCTS_HEADS=lds / SPMCTS_HEADS_C256=lds, in a child process) bit for bit: same
    per-wave k order, same fixed-order cross-wave sums; ragged tails (n % 32) read only live boards; bf16 and
    fp16, C = 128 and 256."""
    from tests.ab_lib import ab_env, product_env, run_child

    run_child(_HEADS_CHILD, ab_env(SPMCTS_HEADS="lds", SPMCTS_HEADS_C256="lds"), tmp_path / "lds.npz")
    run_child(_HEADS_CHILD, product_env(), tmp_path / "co.npz")
    lds, co = np.load(tmp_path / "lds.npz"), np.load(tmp_path / "co.npz")
    assert sorted(lds.files) == sorted(co.files) and len(co.files) == 4 * len(_HEADS_CASES)
    for k in co.files:
        assert np.array_equal(lds[k], co[k]), k
        assert np.isfinite(co[k]).all(), k


@pytest.mark.parametrize("ff", [32, 64])
def test_fp16_bench_nets_finite_and_close(ff):
    """The bench's nets as the bench builds them (ResidualTower(7, 6, 7, 20 blocks, filter_factor 32 /
    64), seed-0 default init, BatchNorm at its init statistics) in the fp16 tower: every output finite
    (no activation overflow in fp16; tests/test_fp16_range.py bounds the activations on the host) and
    within 2x torch fp16 autocast's deviation from the fp32 forward (+2e-3)."""
    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=ff).cuda().eval()
    x = _planes(7, 6, 2048, seed=3)
    with torch.no_grad():
        ref_p, ref_v = net.forward_planes(x)
        with torch.autocast("cuda", dtype=torch.float16):
            ap, av = net.forward_planes(x)
    p, v = HipTowerEvaluator(net, dtype=torch.float16)(x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    assert torch.isfinite(p).all() and torch.isfinite(v).all()
    e_hip = max((p - ref_p).abs().max().item(), (v - ref_v.view(-1)).abs().max().item())
    e_ac = max((ap.float() - ref_p).abs().max().item(), (av.float() - ref_v).abs().max().item())
    assert e_hip <= 2 * e_ac + 2e-3, (e_hip, e_ac)


_RING_CHILD = r"""
import json, sys, torch
sys.path.insert(0, {repo!r})
from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
from tests.test_gpu_tower import _net, _planes
out = {{}}
for dt in (torch.bfloat16, torch.float16):
    net = _net(7, 6, 7, 20, 32)
    x = _planes(7, 6, 999)
    with torch.no_grad():
        rp, rv = net.forward_planes(x)
    hip = HipTowerEvaluator(net, dtype=dt)
    xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    p, v = hip(xb)
    cnt = torch.tensor([999], dtype=torch.int32, device=x.device)
    pd, vd = hip.forward_dev(xb, cnt, 999)
    torch.cuda.synchronize()
    p7, v7 = hip(xb[:7].contiguous(memory_format=torch.channels_last))
    out[str(dt)] = dict(err=max((p - rp).abs().max().item(), (v - rv.view(-1)).abs().max().item()),
                        dev_equal=bool(torch.equal(pd[:999], p) and torch.equal(vd[:999].view(-1), v.view(-1))),
                        batch_equal=bool(torch.equal(p7, p[:7]) and torch.equal(v7, v[:7])))
print(json.dumps(out))
"""


def test_ring_trunk_variant():
    """The LDS weight-ring trunk (csrc/tower_ring.h, SPMCTS_TOWER_RING=1: read once per process, so it
    runs in a child process): the same tolerance against the fp32 forward as the default trunk
    (test_tower_matches_fp32_reference's 0.05 bound), bit-identical device-count and host-count
    outputs, and batch independence.  Measured slower than the default trunk."""
    import json
    import os
    import subprocess
    import sys

    from tests.ab_lib import ab_env

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = ab_env(SPMCTS_TOWER_RING="1")  # the ring trunk is in the A/B library only
    r = subprocess.run([sys.executable, "-c", _RING_CHILD.format(repo=repo)], env=env, capture_output=True, text=True,
                       timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for dt, d in res.items():
        assert d["err"] < 0.05 and d["dev_equal"] and d["batch_equal"], (dt, d)


_WIDE_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from tests.test_gpu_tower import _net, _planes
from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
out = {}
for dt, name in ((torch.bfloat16, "bf16"), (torch.float16, "fp16")):
    hip = HipTowerEvaluator(_net(7, 6, 7, 3, 64), dtype=dt)
    x = _planes(7, 6, 1601).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    p, v = hip(x)
    out["p" + name], out["v" + name] = p.float().cpu().numpy(), v.float().cpu().numpy()
    cnt = torch.tensor([1000], dtype=torch.int32, device="cuda")
    pd, vd = hip.forward_dev(x, cnt, 1601)
    out["pd" + name], out["vd" + name] = pd[:1000].float().cpu().numpy(), vd[:1000].float().cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def test_c256_tile_sets(tmp_path):
    """The C = 256 trunk's tile sets (each in its own process: the switches are read once):
    * the A/B library's 6-board one-buffer 32x32x16 tiles (tower_wide.h, round 4's product trunk,
      SPMCTS_TOWER_C256=32) give every board the same bits as its 3-board tiles (SPMCTS_TOWER_C256=3): host
      batch (full tiles + tails) and the device-count path on a ragged batch, bf16 and fp16;
    * the product library's 16x16x32 one-buffer tiles (tower_wide16.h, its own M16 weight blob) agree with
      them within 1e-2 on probabilities and values (the same products summed in another order; each is
      checked against the fp32 module by test_tower_matches_fp32_reference)."""
    import os
    import subprocess
    import sys

    from tests.ab_lib import ab_env, product_env

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for tiles, env in (("3", ab_env(SPMCTS_TOWER_C256="3")), ("32", ab_env(SPMCTS_TOWER_C256="32")),
                       ("16", product_env())):
        out = tmp_path / f"c{tiles}.npz"
        subprocess.run([sys.executable, "-c", _WIDE_CHILD, root, str(out)], env=env, check=True, timeout=300)
        res[tiles] = np.load(out)
    for k in res["3"].files:
        assert np.array_equal(res["3"][k], res["32"][k]), k
        assert np.abs(res["16"][k].astype(np.float64) - res["32"][k]).max() < 1e-2, k
        assert not np.array_equal(res["16"][k], res["32"][k]), k  # the product really runs the other kernel
