"""The trainer's 3x3 residual-block convolutions on the HIP matrix-core kernels (csrc/trainconv.hip).

The UpdateWorker trains the ResidualTower under fp16 autocast (updateworker.py:147-149), where every
`BasicBlock` conv (games/general/modules.py:13-40) is a conv2d of fp16 activations, weights and bias.
MIOpen runs those as VALU dot2 Winograd kernels (profiles/r04/trainer/); `hip_block_convs(network)`
routes them -- forward, input gradient and weight / bias gradients -- to spmcts_conv3x3_* instead, for
the duration of a `with` block (the trainer's step, eager or while a HIP graph is captured).  Nothing
else of the module changes (no new parameters, the same state_dict), and outside the block the
module's own nn.Conv2d.forward runs again.

Numerics: fp16 operands, fp32 accumulation, one rounding to fp16 per output (as MIOpen's fp16
kernels); the weight gradient is summed over board groups in a fixed order, so results are
deterministic.  Checked against the fp32 torch convolution of the same fp16 operands in
tests/test_gpu_trainconv.py.
"""
import contextlib
import ctypes

import torch

from . import _lib

_F16 = torch.float16


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def supported(width, height, cin, cout):
    return bool(_lib.lib().spmcts_conv3x3_supported(int(width), int(height), int(cin), int(cout)))


def _check(rc, what):
    if rc != 0:
        raise _lib.SpmctsError(f"{what} failed ({rc})")


def conv3x3_forward(x, wf, bias, cout):
    """y = conv(x, w) + fp16(bias) on the packed forward weights wf [cout][9][cin]; x fp16 [n][cin][W][H],
    bias the fp32 parameter (or None)."""
    n, cin, W, H = x.shape
    y = torch.empty((n, cout, W, H), dtype=_F16, device=x.device)
    _check(_lib.lib().spmcts_conv3x3_fwd(n, W, H, cin, cout, _ptr(x), _ptr(wf), _ptr(bias), _ptr(y), _stream()),
           "spmcts_conv3x3_fwd")
    return y


def pack(w):
    """The fp32 weight parameter, rounded to fp16, as (wf [cout][9][cin], wb [cin][9][cout] taps flipped)."""
    w = w.detach().float().contiguous()
    cout, cin = w.shape[:2]
    wf = torch.empty((cout, 9, cin), dtype=_F16, device=w.device)
    wb = torch.empty((cin, 9, cout), dtype=_F16, device=w.device)
    _check(_lib.lib().spmcts_conv3x3_pack(cin, cout, _ptr(w), _ptr(wf), _ptr(wb), _stream()), "spmcts_conv3x3_pack")
    return wf, wb


def weight_grad(x, dy, bias_grad=True):
    """(dw [cout][cin][3][3], db [cout] or None) of y = conv(x, w) + b for the output grad dy: the fp16-rounded
    sums as fp32 tensors (the gradient autocast's fp16 cast hands back to its fp32 parameters)."""
    n, cin, W, H = x.shape
    cout = dy.shape[1]
    splits = (n + 7) // 8  # one slice of 8 boards per partial sum (trainconv.hip k_conv3x3_wgrad)
    part = torch.empty((splits, cout, 9, cin), dtype=torch.float32, device=x.device)
    dw = torch.empty((cout, cin, 3, 3), dtype=torch.float32, device=x.device)
    db = torch.empty((cout,), dtype=torch.float32, device=x.device) if bias_grad else None
    _check(_lib.lib().spmcts_conv3x3_wgrad(n, W, H, cin, cout, _ptr(x), _ptr(dy), _ptr(part), splits, _ptr(dw),
                                           _ptr(db), _stream()), "spmcts_conv3x3_wgrad")
    return dw, db


class Conv3x3(torch.autograd.Function):
    """conv2d(x, w, b, stride 1, padding 1) as autocast runs it: x, w and b rounded to fp16, fp16 output.
    The weight and bias parameters are read in their own dtype (fp32) and rounded inside the kernels, so the
    two cast kernels autocast runs per parameter and direction do not run."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b):
        ctx.dtypes = (x.dtype, w.dtype, None if b is None else b.dtype)
        x = x.to(_F16).contiguous()
        wf, wb = pack(w)
        bias = None if b is None else b.detach().float().contiguous()
        y = conv3x3_forward(x, wf, bias, w.shape[0])
        ctx.save_for_backward(x, wb)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        x, wb = ctx.saved_tensors
        xt, wt, bt = ctx.dtypes
        gy = gy.to(_F16).contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = conv3x3_forward(gy, wb, None, x.shape[1]).to(xt)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            gw, gb = weight_grad(x, gy, ctx.has_bias)
            gw = gw.to(wt)
            gb = None if gb is None else gb.to(bt)
        return gx, gw, gb


def _forward(conv, x):
    return Conv3x3.apply(x, conv.weight, conv.bias)


# Channel counts the trainer routes by default: the ones whose graphed step was timed against MIOpen
# (ResNet-128: 3.26 vs ~5 ms, profiles/r04/trainer/).  The kernels also take C = 256 (checked for
# correctness in tests/test_gpu_trainconv.py), but there k_conv3x3 holds its whole A operand in registers
# (9 x 8 f16x8 = 288 VGPRs) and spills, and no step A/B exists: channels=(128, 256) opts in.
MEASURED_CHANNELS = (128,)


@contextlib.contextmanager
def hip_block_convs(network, enabled=True, channels=MEASURED_CHANNELS):
    """Within the block, the residual blocks' 3x3 convolutions of `network` (a ResidualTower on a CUDA
    device, run under fp16 autocast) go through Conv3x3.  Yields whether they do (False: unsupported
    shape or padding mode, a channel count outside `channels`, another module type, or not enabled --
    the module's own convolutions run)."""
    blocks = getattr(network, "residual_blocks", None)
    convs = [] if blocks is None else [c for blk in blocks for c in (blk.conv1, blk.conv2)]
    ok = (enabled and convs and all(
        isinstance(c, torch.nn.Conv2d) and c.kernel_size == (3, 3) and c.stride == (1, 1) and c.padding == (1, 1)
        and c.padding_mode == "zeros" and c.groups == 1 and c.dilation == (1, 1) and c.weight.is_cuda
        and c.in_channels in channels and c.out_channels in channels for c in convs)
        and all(supported(network.width, network.height, c.in_channels, c.out_channels) for c in convs))
    if not ok:
        yield False
        return
    for c in convs:
        c.forward = (lambda x, c=c: _forward(c, x))
    try:
        yield True
    finally:
        for c in convs:
            del c.forward
