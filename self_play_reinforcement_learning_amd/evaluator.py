"""Leaf evaluators: turn the arena's leaf rows into (priors, values) on the same stream.

The reference calls `network(state, player)` once per expansion, over a
multiprocessing queue when proxied (games/algos/inference_proxy.py:21-24,
inference_worker.py:100-119).  Here every pending leaf of every tree arrives
as one device tensor and the network runs once per simulation step.

Supported networks (chosen in `make_evaluator`):
  * `ResidualTower` (this package or any module with `forward_planes`): a frozen
    BatchNorm-folded bf16 channels_last `InferenceTower` reads the encoded
    planes directly;
  * `DeviceTableNet`: the deterministic table network kernel (parity tests);
  * any other `nn.Module` with the reference's `forward(boards[B, W, H])`;
  * any other callable with the reference's `net(state, player)` protocol —
    evaluated row by row (a compatibility path for e.g. InferenceProxy-like
    objects, not a throughput path).
"""
import logging
import numpy as np
import torch
from torch import nn

from .arena import GAMES, table_net_eval
from .modules import InferenceTower


class DeviceTableNet:
    """Deterministic network (identical to oracle/table_net.py) evaluated by a HIP kernel."""

    def __init__(self, game="connect4", salt=0):
        self.game = game
        self.salt = salt
        _, self.width, self.height, self.n_actions = GAMES[game]

    def to(self, *a, **k):
        return self

    def train(self, *a, **k):
        return self

    def eval(self):
        return self

    def share_memory(self):
        return self

    def forward_leaves(self, leaves, leaf_format, leaf_layout):
        return table_net_eval(self.game, leaves, leaf_format, leaf_layout, self.salt)

    def __call__(self, state, player=1):
        s = torch.as_tensor(np.asarray(state) * player, dtype=torch.int64).reshape(1, self.width, self.height)
        probs, v = self.forward_leaves(s.cuda(), "board", "nchw")
        return probs[0].tolist(), float(v[0]) * player


class Evaluator:
    """callable(leaves [n, ...]) -> (probs f32 [n, A] contiguous, values f32 [n]).

    `snapshot`: the evaluator reads its own copy of the weights (refreshed by refresh()), never the
    live module's parameters / BatchNorm buffers, so optimizer steps on another stream may run beside
    its evaluations (SelfPlayScheduler's overlapped trainer); False = it reads the live module."""

    leaf_format = "bf16"
    leaf_layout = "nchw"
    snapshot = False

    def empty_root_input(self, W, H, device):
        """The input row of the empty board (`network(base_state)`, mcts.py:167-168)."""
        if self.leaf_format == "board":
            return torch.zeros((1, W, H), dtype=torch.int64, device=device)
        dt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[self.leaf_format]
        x = torch.zeros((1, 3, W, H), dtype=dt, device=device)
        x[:, 0] = 1
        if self.leaf_layout == "nhwc":
            x = x.contiguous(memory_format=torch.channels_last)
        return x


class TableEvaluator(Evaluator):
    snapshot = True  # no trainable weights

    def __init__(self, net, leaf_format="f32", leaf_layout="nchw"):
        self.net = net
        self.leaf_format, self.leaf_layout = leaf_format, leaf_layout

    def __call__(self, leaves):
        return self.net.forward_leaves(leaves, self.leaf_format, self.leaf_layout)


class TowerEvaluator(Evaluator):
    """InferenceTower on encoded planes (bf16 by default)."""

    def __init__(self, tower, dtype=torch.bfloat16, leaf_layout="nhwc", device=None):
        self.tower = tower
        self.dtype = dtype
        self.leaf_format = {torch.bfloat16: "bf16", torch.float16: "f16", torch.float32: "f32"}[dtype]
        self.leaf_layout = leaf_layout
        self.device = device
        self.refresh()

    @property
    def snapshot(self):
        # bf16 / fp16 folding copies every tensor; in fp32 `.to(float32)` can alias the live bias and
        # linear_output tensors
        return self.dtype != torch.float32

    @torch.no_grad()
    def refresh(self):
        """Re-fold the weights after the source tower changed (epoch boundary)."""
        src = self.tower
        if self.device is not None:
            src = src.to(self.device)
        was_training = src.training
        src.eval()
        self.inf = InferenceTower(src, dtype=self.dtype)
        src.train(was_training)

    @torch.no_grad()
    def __call__(self, leaves):
        probs, value = self.inf.forward_planes(leaves)
        return probs.contiguous(), value.reshape(-1).float().contiguous()


class ModuleEvaluator(Evaluator):
    """Any nn.Module with the reference's batched `forward(boards)` (modules.py:88-107)."""

    leaf_format = "board"

    def __init__(self, module):
        self.module = module

    @torch.no_grad()
    def __call__(self, leaves):
        probs, value = self.module.forward(leaves)
        return probs.float().contiguous(), value.reshape(-1).float().contiguous()


class CallableEvaluator(Evaluator):
    """Row-by-row `net(state, player)` (the reference protocol) for arbitrary callables."""

    leaf_format = "board"

    def __init__(self, fn, n_actions):
        self.fn = fn
        self.n_actions = n_actions

    def __call__(self, leaves):
        boards = leaves.cpu().numpy()
        probs = np.zeros((len(boards), self.n_actions), dtype=np.float32)
        values = np.zeros(len(boards), dtype=np.float32)
        for i, b in enumerate(boards):
            p, v = self.fn(b, 1)
            probs[i] = p
            values[i] = v
        return torch.as_tensor(probs).to(leaves.device), torch.as_tensor(values).to(leaves.device)


def make_evaluator(network, game, device=None, dtype=torch.bfloat16, leaf_layout="nhwc", backend="auto"):
    """backend: "auto" (fused HIP trunk when instantiated for the net, else torch), "hip", "torch"."""
    _, W, H, A = GAMES[game]
    if isinstance(network, Evaluator):
        return network
    if isinstance(network, DeviceTableNet):
        return TableEvaluator(network)
    if isinstance(network, nn.Module) and hasattr(network, "residual_blocks") and hasattr(network, "conv_policy"):
        if device is not None:
            network.to(device)
        if backend == "hip" or (backend == "auto" and dtype in (torch.bfloat16, torch.float16)
                                and HipTowerEvaluator.supported(network)):
            return HipTowerEvaluator(network, device=device, dtype=dtype)
        if backend == "auto":
            logging.getLogger(__name__).info(
                "fused HIP tower not instantiated for %s x %s boards with %d channels (built: 7x6 / 3x3, C = 128 or "
                "256): leaf evaluation runs on the PyTorch TowerEvaluator (MIOpen convolutions, %s)",
                W, H, 4 * int(getattr(network, "filter_factor", 0)), dtype)
        return TowerEvaluator(network, dtype=dtype, leaf_layout=leaf_layout, device=device)
    if isinstance(network, nn.Module):
        if device is not None:
            network.to(device)
        network.eval()
        return ModuleEvaluator(network)
    if callable(network):
        return CallableEvaluator(network, A)
    raise TypeError(f"cannot evaluate leaves with {type(network).__name__}")


# ----------------------------------------------------------------------------- fused HIP tower
def phys_channel_order(c):
    """Logical channel held at each PHYSICAL LDS position of the fused tower's activations
    (csrc/tower.hip phys_off): within every 32-channel tile, position 16h + 4g + j holds the MFMA
    output row 8g + 4h + j."""
    p = torch.arange(c)
    w = p % 32
    return (p - w) + 8 * ((w % 16) // 4) + 4 * (w // 16) + w % 4


def phys_channel_order_m16(c):
    """The phys16 order of the 16x16x32 trunk (csrc/tower_m16.h): within every 64-channel half, physical
    position 16 q + 4 m + r holds output channel 16 m + 4 q + r (a lane's four 16-channel tiles' values
    of one cell are one contiguous run).  The map swaps q and m, so it is its own inverse."""
    p = torch.arange(c)
    w = p % 64
    return (p - w) + 16 * ((w % 16) // 4) + 4 * (w // 16) + w % 4


def _pack_conv_m16(w, dtype=torch.bfloat16):
    """A block conv for the 16x16x32 trunk (csrc/tower_m16.h): [Cout][Cin][3][3] -> fragments
    [Cout/16][taps][Cin/32][64 lanes][8], lane 16 q + n holding W[16 ct + n][tap][physical input channels
    32 k + 8 q .. + 8] (the input channel axis in the phys16 order of the layer that wrote them)."""
    cout, cin, kh, kw = w.shape
    w = w[:, phys_channel_order_m16(cin).to(w.device)]
    taps = kh * kw
    w = w.permute(0, 2, 3, 1).reshape(cout, taps, cin)               # [o][tap][c]
    w = w.reshape(cout // 16, 16, taps, cin // 32, 4, 8)             # o = ct*16 + n ; c = k*32 + q*8 + j
    w = w.permute(0, 2, 3, 4, 1, 5)                                  # [ct][tap][k][q][n][j] -> lane = q*16 + n
    return w.reshape(-1).to(dtype)


def _pack_conv(w, cin_pad=None, in_perm=False, dtype=torch.bfloat16, order=None):
    """[Cout][Cin][kh][kw] fp -> bf16 / fp16 fragments [Cout/32][taps][Cin/16][64 lanes][8] (csrc/tower.hip).
    in_perm: the layer reads activations another tower layer wrote, which sit in the physical channel
    order (phys_channel_order), so the input-channel axis is permuted to match."""
    cout, cin, kh, kw = w.shape
    if in_perm:
        w = w[:, (order or phys_channel_order)(cin).to(w.device)]
    if cin_pad is not None and cin_pad > cin:
        w = torch.cat([w, torch.zeros(cout, cin_pad - cin, kh, kw, dtype=w.dtype, device=w.device)], 1)
        cin = cin_pad
    taps = kh * kw
    w = w.permute(0, 2, 3, 1).reshape(cout, taps, cin)               # [o][tap][c], tap = i*3 + j
    w = w.reshape(cout // 32, 32, taps, cin // 16, 2, 8)             # o = ct*32 + r ; c = kk*16 + h*8 + j
    w = w.permute(0, 2, 3, 4, 1, 5)                                  # [ct][tap][kk][h][r][j] -> lane = h*32 + r
    return w.reshape(-1).to(dtype)


class HipTowerEvaluator(Evaluator):
    """ResidualTower leaf evaluation on the fused HIP trunk kernel (csrc/tower.hip).

    The stem, every BasicBlock and the two 1x1 head convs run in one launch with
    the activations resident in LDS; the three small linear heads (policy
    1344->A + softmax, value 1344->8ff->1 + tanh) run in the fused MFMA heads kernel.
    dtype: the weights' / activations' / head features' element type, torch.bfloat16 or
    torch.float16 (the reference's inference dtype: amp.autocast, inference_worker.py:117); fp32
    accumulation, fp32 biases, bf16 0/1 leaf planes either way.
    """

    @property
    def pure_planes(self):
        """With the MFMA heads kernel a board's outputs depend only on its planes, bit for bit
        whatever batch it is in (tests/test_gpu_tower.py): duplicate leaves of a batch may share one
        row (SelfPlayEngine leaf_dedup).  The torch-GEMM heads are not batch-independent."""
        return self.fused_heads is True

    leaf_format = "bf16"
    leaf_layout = "nhwc"
    bucket = 1  # the HIP kernels take any batch size; no shape padding needed
    snapshot = True  # packed weight / bias blobs (refresh())

    def __init__(self, tower, device=None, fused_heads=True, dtype=torch.bfloat16):
        """fused_heads: True = MFMA heads kernel (deterministic, batch-independent), "gemm" =
        one hipBLASLt GEMM + epilogue kernel, False = torch ops in `dtype`."""
        from . import _lib

        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError(f"fused tower dtype must be bfloat16 or float16, not {dtype}")
        self.dtype = dtype
        self.flags = _lib.TOWER_F16 if dtype == torch.float16 else 0
        self.fused_heads = fused_heads
        self._lib = _lib
        self.tower = tower
        self.device = device
        self.C = 4 * tower.filter_factor
        self.W, self.H, self.A = tower.width, tower.height, tower.action_size
        if not _lib.lib().spmcts_tower_supported(self.W, self.H, self.C):
            raise ValueError(f"fused tower not instantiated for {self.W}x{self.H} boards, {self.C} channels")
        self.refresh()

    def set_dtype(self, dtype):
        """Repack the weights for the other trunk element type (bf16 <-> fp16) and drop the device
        buffers (reallocated at the next forward); the caller refreshes its root prior
        (SelfPlayEngine.refresh_network)."""
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError(f"fused tower dtype must be bfloat16 or float16, not {dtype}")
        self.dtype = dtype
        self.flags = self._lib.TOWER_F16 if dtype == torch.float16 else 0
        self._dev_bufs = None
        self.refresh()

    @staticmethod
    def supported(tower):
        from . import _lib

        C = 4 * getattr(tower, "filter_factor", 0)
        return bool(_lib.lib().spmcts_tower_supported(tower.width, tower.height, C))

    @torch.no_grad()
    def refresh(self):
        t = self.tower
        dev = self.device if self.device is not None else next(t.parameters()).device
        was = t.training
        t.eval()
        fold = InferenceTower._fold
        ws, bs = [], []
        w, b = fold(t.conv1, t.bn1)
        dt = self.dtype
        # the blob layout the library's trunk for this shape expects (include/spmcts.h SPMCTS_WLAYOUT_*)
        self.wlayout = self._lib.lib().spmcts_tower_weight_layout(self.W, self.H, self.C)
        m16 = self.wlayout == self._lib.WLAYOUT_M16
        ws.append(_pack_conv(w, cin_pad=16, dtype=dt))
        bs.append(b)
        for blk in t.residual_blocks:
            for conv, bn in ((blk.conv1, blk.bn1), (blk.conv2, blk.bn2)):
                w, b = fold(conv, bn)
                ws.append(_pack_conv_m16(w, dtype=dt) if m16 else _pack_conv(w, in_perm=True, dtype=dt))
                bs.append(b)
        wp, bp = fold(t.conv_policy, t.policy_bn)
        wv, bv = fold(t.conv_value, t.value_bn)
        ws.append(_pack_conv(torch.cat([wp, wv], 0), in_perm=True, dtype=dt,
                             order=phys_channel_order_m16 if m16 else phys_channel_order))
        bs.append(torch.cat([bp, bv], 0))
        self.n_blocks = len(t.residual_blocks)
        self.wblob = torch.cat(ws).to(dev).contiguous()
        self.bblob = torch.cat([x.float() for x in bs]).to(dev).contiguous()
        ff, cells = t.filter_factor, self.W * self.H

        def nhwc_cols(lin):
            m = lin.weight.detach()
            return m.view(m.shape[0], ff, self.W, self.H).permute(0, 2, 3, 1).reshape(m.shape[0], -1)

        bf = self.dtype
        self.lp_w = nhwc_cols(t.linear_policy).to(dev, bf).contiguous()
        self.lp_b = t.linear_policy.bias.detach().to(dev, bf)
        self.fv_w = nhwc_cols(t.fc_value).to(dev, bf).contiguous()
        self.fv_b = t.fc_value.bias.detach().to(dev, bf)
        self.lo_w = t.linear_output.weight.detach().to(dev, bf)
        self.lo_b = t.linear_output.bias.detach().to(dev, bf)
        self.ff, self.cells = ff, cells
        # fused-heads blobs (csrc/tower.hip k_heads)
        K = cells * ff
        wp = torch.zeros(32, K, dtype=bf, device=dev)
        wp[: self.A] = self.lp_w
        # fragment swizzle: tile j (0 = policy padded to 32 rows, 1.. = value hidden rows), k-step s,
        # lane (r, h) -> W[32 j + r][16 s + 8 h .. + 8]: one contiguous KiB per (tile, k-step)
        wall = torch.cat([wp, self.fv_w], 0)
        nt, ks = wall.shape[0] // 32, K // 16
        self.head_w = wall.view(nt, 32, ks, 2, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(-1)
        bp = torch.zeros(32, dtype=torch.float32, device=dev)
        bp[: self.A] = t.linear_policy.bias.detach().float().to(dev)
        self.head_b = torch.cat([bp, t.fc_value.bias.detach().float().to(dev),
                                 t.linear_output.weight.detach().float().reshape(-1).to(dev),
                                 t.linear_output.bias.detach().float().reshape(-1).to(dev)]).contiguous()
        # GEMM-heads blobs: Wc [hidden + A (padded to 16)][cells * 2ff] over the interleaved features
        hid = 8 * ff
        npad = -(-(hid + self.A) // 16) * 16
        wc = torch.zeros(npad, cells, 2 * ff, dtype=torch.float32, device=dev)
        wc[:hid, :, ff:] = nhwc_cols(t.fc_value).float().view(hid, cells, ff)
        wc[hid:hid + self.A, :, :ff] = nhwc_cols(t.linear_policy).float().view(self.A, cells, ff)
        self.wc = wc.reshape(npad, -1).to(bf).contiguous()
        self.hid = hid
        self.epi_b = torch.cat([t.fc_value.bias.detach().float(), t.linear_output.weight.detach().float().reshape(-1),
                                t.linear_output.bias.detach().float().reshape(-1),
                                t.linear_policy.bias.detach().float()]).to(dev).contiguous()
        t.train(was)

    supports_device_count = True
    # set by engine.LanedEngine: the tower launches share the chip with other lanes' launches, so
    # tiles are packed full (SPMCTS_TOWER_PACK) instead of aligned to whole chip rounds
    concurrent = False

    def reserve(self, rows, device):
        """(Re)allocate the device-count path's output buffers for at least `rows` rows."""
        buf = getattr(self, "_dev_bufs", None)
        if buf is None or buf[0].shape[0] < rows or buf[0].device != device:
            self._dev_bufs = (torch.empty((rows, self.cells, self.C // 2), dtype=self.dtype, device=device),
                              torch.empty((rows, self.A), dtype=torch.float32, device=device),
                              torch.empty(rows, dtype=torch.float32, device=device))

    @torch.no_grad()
    def forward_dev(self, leaves, count_dev, max_rows):
        """Evaluate the first *count_dev rows of `leaves` without a host synchronisation.

        leaves: the arena's whole leaf buffer (NCHW view of NHWC bf16 storage, >= max_rows rows);
        count_dev: device int32 holding the row count.  Returns max_rows-row probs/values buffers
        of which the first *count_dev rows are valid (the arena's expand reads the same count)."""
        self.tower_dev(leaves, count_dev, max_rows)
        return self.heads_dev(count_dev, max_rows)

    def tower_dev(self, leaves, count_dev, max_rows):
        """The trunk half of forward_dev (k_tower_dyn) on the current stream."""
        dev = leaves.device
        self.reserve(max_rows, dev)
        feats, probs, values = self._dev_bufs
        c = self._lib.ctypes.c_void_p
        stream = c(torch.cuda.current_stream().cuda_stream)
        L = self._lib.lib()
        timer = getattr(self, "tower_timer", None)
        if timer is not None:
            timer.start()
        flags = (self._lib.TOWER_PACK if self.concurrent else 0) | self.flags
        rc = L.spmcts_tower_forward_dev(self.W, self.H, self.C, self.n_blocks, c(leaves.data_ptr()),
                                        c(count_dev.data_ptr()), max_rows, c(self.wblob.data_ptr()),
                                        c(self.bblob.data_ptr()), c(feats.data_ptr()), flags, stream)
        if timer is not None:
            timer.stop()
        if rc != 0:
            raise self._lib.tower_error("spmcts_tower_forward_dev", rc)

    def heads_dev(self, count_dev, max_rows):
        """The linear-heads half of forward_dev (k_heads) on the current stream."""
        feats, probs, values = self._dev_bufs
        c = self._lib.ctypes.c_void_p
        stream = c(torch.cuda.current_stream().cuda_stream)
        rc = self._lib.lib().spmcts_tower_heads_dev(self.W, self.H, self.C, self.A, c(feats.data_ptr()),
                                                    c(count_dev.data_ptr()), max_rows, c(self.head_w.data_ptr()),
                                                    c(self.head_b.data_ptr()), c(probs.data_ptr()),
                                                    c(values.data_ptr()), self.flags, stream)
        if rc != 0:
            raise self._lib.tower_error("spmcts_tower_heads_dev", rc)
        return probs, values

    @torch.no_grad()
    def trunk(self, planes_nhwc):
        """planes: bf16 [n, W, H, 3] contiguous -> head features [n, cells, C/2] in self.dtype."""
        n = planes_nhwc.shape[0]
        feats = torch.empty((max(n, 1), self.cells, self.C // 2), dtype=self.dtype, device=planes_nhwc.device)
        if n:
            stream = torch.cuda.current_stream().cuda_stream
            rc = self._lib.lib().spmcts_tower_forward(
                self.W, self.H, self.C, self.n_blocks, self._lib.ctypes.c_void_p(planes_nhwc.data_ptr()), n,
                self._lib.ctypes.c_void_p(self.wblob.data_ptr()), self._lib.ctypes.c_void_p(self.bblob.data_ptr()),
                self._lib.ctypes.c_void_p(feats.data_ptr()), self.flags, self._lib.ctypes.c_void_p(stream))
            if rc != 0:
                raise self._lib.tower_error("spmcts_tower_forward", rc)
        return feats[:n]

    @torch.no_grad()
    def __call__(self, leaves):
        # leaves: NCHW view over NHWC storage (arena leaf buffer) or any [n, 3, W, H] planes
        planes = leaves.permute(0, 2, 3, 1)
        if planes.dtype != torch.bfloat16 or not planes.is_contiguous():
            planes = planes.to(torch.bfloat16).contiguous()
        n = planes.shape[0]
        f = self.trunk(planes)
        if self.fused_heads == "gemm":
            z = torch.matmul(f.reshape(n, -1), self.wc.t()).to(torch.bfloat16)  # one GEMM for both heads
            probs = torch.empty((max(n, 1), self.A), dtype=torch.float32, device=f.device)
            value = torch.empty(max(n, 1), dtype=torch.float32, device=f.device)
            if n:
                c = self._lib.ctypes.c_void_p
                rc = self._lib.lib().spmcts_head_epilogue(
                    self.hid, self.A, c(z.data_ptr()), z.shape[1], n, c(self.epi_b.data_ptr()), c(probs.data_ptr()),
                    c(value.data_ptr()), c(torch.cuda.current_stream().cuda_stream))
                if rc != 0:
                    raise self._lib.tower_error("spmcts_head_epilogue", rc)
            return probs[:n], value[:n]
        if self.fused_heads:
            probs = torch.empty((max(n, 1), self.A), dtype=torch.float32, device=f.device)
            value = torch.empty(max(n, 1), dtype=torch.float32, device=f.device)
            if n:
                c = self._lib.ctypes.c_void_p
                rc = self._lib.lib().spmcts_tower_heads(
                    self.W, self.H, self.C, self.A, c(f.data_ptr()), n, c(self.head_w.data_ptr()),
                    c(self.head_b.data_ptr()), c(probs.data_ptr()), c(value.data_ptr()), self.flags,
                    c(torch.cuda.current_stream().cuda_stream))
                if rc != 0:
                    raise self._lib.tower_error("spmcts_tower_heads", rc)
            return probs[:n], value[:n]
        pf = f[:, :, : self.ff].reshape(n, -1)
        vf = f[:, :, self.ff:].reshape(n, -1)
        probs = torch.softmax(torch.nn.functional.linear(pf, self.lp_w, self.lp_b).float(), dim=1)
        v = torch.relu(torch.nn.functional.linear(vf, self.fv_w, self.fv_b))
        value = torch.tanh(torch.nn.functional.linear(v, self.lo_w, self.lo_b).float()).reshape(-1)
        return probs.contiguous(), value.contiguous()
