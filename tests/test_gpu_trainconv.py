"""GPU: the trainer's 3x3 convolutions on the HIP matrix-core kernels (csrc/trainconv.hip, trainconv.py)
against torch's fp32 convolution of the same fp16 operands.

The reference trains under fp16 autocast (updateworker.py:147-149), where each residual-block conv
(games/general/modules.py:13-40) is conv2d(x16, w16, b16).  Tolerances (stated): forward output and input
gradient within 2e-3 x max|ref| (fp32 accumulation of fp16 products, one fp16 rounding of the output);
weight and bias gradients within 2e-3 x max|ref| (sums over 64 boards x the cells, rounded to fp16 once).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x, w, b, gy):
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    y = torch.nn.functional.conv2d(xr, wr, br, padding=1)
    y.backward(gy.float())
    return y.detach(), xr.grad, wr.grad, br.grad


def _close(got, ref, tol=2e-3):
    scale = ref.abs().max().item()
    err = (got.float() - ref).abs().max().item()
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("W,H,cin,cout,n", [(7, 6, 128, 128, 64), (7, 6, 256, 256, 16), (3, 3, 128, 128, 64),
                                            (7, 6, 128, 128, 5)])
def test_conv3x3_matches_torch(W, H, cin, cout, n):
    from self_play_reinforcement_learning_amd.trainconv import Conv3x3, supported

    assert supported(W, H, cin, cout)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, cin, W, H, device="cuda", generator=g).half()
    w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.05).half()
    b = (torch.randn(cout, device="cuda", generator=g) * 0.1).half()
    gy = torch.randn(n, cout, W, H, device="cuda", generator=g).half()
    yr, gxr, gwr, gbr = _ref(x, w, b, gy)
    xs, ws, bs = (t.clone().requires_grad_(True) for t in (x, w, b))
    with torch.autocast("cuda", dtype=torch.float16):
        y = Conv3x3.apply(xs, ws, bs)
    assert y.dtype == torch.float16 and y.shape == (n, cout, W, H)
    y.backward(gy)
    _close(y, yr)
    _close(xs.grad, gxr)
    _close(ws.grad, gwr)
    _close(bs.grad, gbr)
    # deterministic: a second run gives the same bits
    xs2, ws2, bs2 = (t.clone().requires_grad_(True) for t in (x, w, b))
    with torch.autocast("cuda", dtype=torch.float16):
        y2 = Conv3x3.apply(xs2, ws2, bs2)
    y2.backward(gy)
    assert torch.equal(y, y2) and torch.equal(xs.grad, xs2.grad) and torch.equal(ws.grad, ws2.grad)
    assert torch.equal(bs.grad, bs2.grad)


def test_hip_block_convs_patch_is_scoped():
    """hip_block_convs routes exactly the residual blocks' 3x3 convs and restores the modules afterwards;
    unsupported shapes (C = 64) leave the module's own convolutions in place."""
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.trainconv import hip_block_convs

    net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=32).cuda().eval()  # no dropout masks
    keys = list(net.state_dict())
    x = torch.randint(-1, 2, (8, 7, 6), device="cuda")
    with torch.autocast("cuda", dtype=torch.float16):
        p0, v0 = net.forward(x)
        with hip_block_convs(net) as on:
            assert on and "forward" in vars(net.residual_blocks[0].conv1)
            p1, v1 = net.forward(x)
        assert "forward" not in vars(net.residual_blocks[0].conv1)
    assert list(net.state_dict()) == keys
    assert (p0.float() - p1.float()).abs().max() < 1e-2 and (v0.float() - v1.float()).abs().max() < 1e-2
    small = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=16).cuda()
    with hip_block_convs(small) as on:
        assert not on
    # C = 256 runs only when asked for (no step A/B against MIOpen at that width, trainconv.MEASURED_CHANNELS)
    wide = ResidualTower(7, 6, 7, num_blocks=1, filter_factor=64).cuda()
    with hip_block_convs(wide) as on:
        assert not on
    with hip_block_convs(wide, channels=(128, 256)) as on:
        assert on
    # the kernels zero-pad: a conv with another padding mode keeps its own forward
    net.residual_blocks[1].conv2.padding_mode = "reflect"
    with hip_block_convs(net) as on:
        assert not on and "forward" not in vars(net.residual_blocks[0].conv1)


def test_trainer_hip_convs_match_miopen_step():
    """One autocast SGD step of ResNet-128x4 with the HIP block convolutions vs MIOpen's (eval-mode dropout,
    the same batch and weights): the loss within 0.5 %, the weight update pointing the same way (cosine of
    the deltas > 0.99); then captured-graph steps with the HIP convolutions replay deterministically."""
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

    g = torch.Generator().manual_seed(3)
    rows = dict(state=torch.randint(-1, 2, (256, 42), dtype=torch.int8, generator=g),
                tree_probs=torch.softmax(torch.randn(256, 7, generator=g), 1),
                q=torch.rand(256, dtype=torch.float64, generator=g) - 0.5,
                z=torch.randint(-1, 2, (256,), generator=g).float())
    loss, delta, batch = {}, {}, None
    for hip in (False, True):
        torch.manual_seed(0)
        net = ResidualTower(7, 6, 7, num_blocks=4, filter_factor=32).cuda()
        w0 = torch.cat([p.detach().reshape(-1).clone() for p in net.parameters()])
        tr = _Trainer(net, torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9), memory_size=1000, batch_size=64,
                      min_memory=0, q_average=True, device="cuda", overlap=False, autocast=True, train_mode=False,
                      hip_convs=hip)
        assert tr.hip_convs is hip
        tr.memory.add_moves(rows)
        if batch is None:
            batch = tr.memory.sample_batch(64)
        loss[hip] = tr.train_batch(*batch)
        delta[hip] = torch.cat([p.detach().reshape(-1) for p in net.parameters()]) - w0
    assert math.isfinite(loss[True]) and abs(loss[True] - loss[False]) < 5e-3 * abs(loss[False]), loss
    cos = torch.nn.functional.cosine_similarity(delta[True].double(), delta[False].double(), dim=0).item()
    assert cos > 0.99, cos
    # graphed steps (3 eager, capture, replays) with the HIP convolutions: two runs, the same weights (MIOpen's
    # remaining kernels -- stem, heads, batch norm -- asked for deterministic algorithms)
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        out = _graphed_runs(rows)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    assert out[0][0] == out[1][0]
    for k in out[0][1]:
        assert torch.equal(out[0][1][k], out[1][1][k]), k


def _graphed_runs(rows):
    from self_play_reinforcement_learning_amd.modules import ResidualTower
    from self_play_reinforcement_learning_amd.self_play_parallel import _Trainer

    out = []
    for _ in range(2):
        torch.manual_seed(0)
        net = ResidualTower(7, 6, 7, num_blocks=2, filter_factor=32).cuda()
        tr = _Trainer(net, torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9), memory_size=1000, batch_size=64,
                      min_memory=0, q_average=True, device="cuda", overlap=False, autocast=True, train_mode=False,
                      graph=True)
        tr.memory.add_moves(rows)
        torch.manual_seed(5)
        ls = [float(tr._step_graphed(*tr.memory.sample_batch(64))) for _ in range(6)]
        torch.cuda.synchronize()
        assert tr.graph_captures == 1 and all(math.isfinite(v) for v in ls)
        assert tr.hip_convs
        out.append((ls, {k: v.clone() for k, v in net.state_dict().items()}))
    return out
