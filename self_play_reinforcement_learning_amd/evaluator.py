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
    """callable(leaves [n, ...]) -> (probs f32 [n, A] contiguous, values f32 [n])."""

    leaf_format = "bf16"
    leaf_layout = "nchw"

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


def make_evaluator(network, game, device=None, dtype=torch.bfloat16, leaf_layout="nhwc"):
    _, W, H, A = GAMES[game]
    if isinstance(network, Evaluator):
        return network
    if isinstance(network, DeviceTableNet):
        return TableEvaluator(network)
    if isinstance(network, nn.Module) and hasattr(network, "residual_blocks") and hasattr(network, "conv_policy"):
        return TowerEvaluator(network, dtype=dtype, leaf_layout=leaf_layout, device=device)
    if isinstance(network, nn.Module):
        if device is not None:
            network.to(device)
        network.eval()
        return ModuleEvaluator(network)
    if callable(network):
        return CallableEvaluator(network, A)
    raise TypeError(f"cannot evaluate leaves with {type(network).__name__}")
