"""Policy/value ResNet with the reference's exact parameter layout.

`ResidualTower` keeps the constructor signature, module names and parameter
creation order of games/general/modules.py:43-112 (`BasicBlock` :13-40), so

  * `state_dict()` keys/shapes are identical ({"model": state_dict} checkpoints
    written by the reference's UpdateWorker load unchanged);
  * under the same `torch.manual_seed`, random init is bit-identical (same
    nn.Conv2d/nn.Linear construction order, then xavier-uniform + bias 0.01 on
    every Conv2d, rl_utils/weights.py:5-8).

What is new is the inference side used by the arena:
`forward_planes(planes)` consumes the [B, 3, W, H] (empty, own, enemy) planes
the HIP encode kernel writes straight into device memory, skipping the
reference's per-call `preprocess` (modules.py:115-125), and
`InferenceTower` is a frozen, BatchNorm-folded, channels_last bf16 copy for
the leaf-evaluation hot loop.
"""
import torch
from torch import nn
from torch.nn import functional as F


def init_weights(m):
    """rl_utils/weights.py:5-8: xavier-uniform weights, bias 0.01, Conv2d only."""
    if type(m) == nn.Conv2d:
        torch.nn.init.xavier_uniform_(m.weight)
        m.bias.data.fill_(0.01)


def _same(size, kernel_size=3, stride=1, padding=1):
    return (size + padding * 2 - (kernel_size - 1) - 1) // stride + 1


class BasicBlock(nn.Module):
    """Residual block: conv3x3-BN-ReLU-conv3x3-BN (+x) ReLU (modules.py:13-40)."""

    expansion = 1

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=3, stride=stride, padding=1, bias=True)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=True)
        self.bn2 = nn.BatchNorm2d(planes)
        self.stride = stride

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + x)


def planes_from_boards(s, width, height):
    """preprocess (modules.py:115-125): [B, W, H] boards (+1 own) -> float [B, 3, W, H]."""
    s = torch.as_tensor(s)
    s = s.reshape(-1, width, height)
    return torch.stack([(s == 0), (s == 1), (s == -1)], 1).float()


class ResidualTower(nn.Module):
    """ResidualTower(width, height, action_size, num_blocks, default_kernel_size, filter_factor)."""

    def __init__(self, width=7, height=6, action_size=7, num_blocks=15, default_kernel_size=3, filter_factor=32):
        super().__init__()
        self.inplanes = filter_factor * 4
        self.width = width
        self.height = height
        self.action_size = action_size
        self.num_blocks = num_blocks
        self.filter_factor = filter_factor
        k = default_kernel_size
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=k, stride=1, padding=1, bias=True)
        self.bn1 = nn.BatchNorm2d(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        channels = filter_factor * 4
        blocks = [BasicBlock(self.inplanes, channels)]
        self.inplanes = channels
        blocks += [BasicBlock(self.inplanes, channels) for _ in range(1, num_blocks)]
        self.residual_blocks = nn.Sequential(*blocks)
        cells = _same(_same(_same(_same(width))), 1, 1, 0) * _same(_same(_same(_same(height))), 1, 1, 0)
        self.conv_policy = nn.Conv2d(self.inplanes, filter_factor, kernel_size=1, stride=1)
        self.policy_bn = nn.BatchNorm2d(filter_factor)
        self.policy_dropout = nn.Dropout(p=0.5)
        self.linear_policy = nn.Linear(cells * filter_factor, action_size)
        self.softmax = nn.Softmax(dim=1)
        self.conv_value = nn.Conv2d(self.inplanes, filter_factor, kernel_size=1, stride=1)
        self.value_bn = nn.BatchNorm2d(filter_factor)
        self.value_dropout = nn.Dropout(p=0.5)
        self.fc_value = nn.Linear(cells * filter_factor, filter_factor * 8)
        self.linear_output = nn.Linear(filter_factor * 8, 1)
        self.apply(init_weights)

    @staticmethod
    def from_env(env, num_blocks=15, filter_factor=32):
        """modules.py:75-77"""
        return ResidualTower(env.width, env.height, env.num_actions(), num_blocks, filter_factor=filter_factor)

    def forward_planes(self, x):
        x = self.relu(self.bn1(self.conv1(x)))
        x = self.residual_blocks(x)
        policy = F.relu(self.policy_bn(self.conv_policy(x))).flatten(1)
        policy = self.softmax(self.linear_policy(self.policy_dropout(policy)))
        value = F.relu(self.value_bn(self.conv_value(x))).flatten(1)
        value = F.relu(self.fc_value(self.value_dropout(value)))
        value = torch.tanh(self.linear_output(value))
        return policy, value

    def forward(self, x):
        """Reference protocol: [B, W, H] boards (own = +1) -> (probs [B, A], value [B, 1])."""
        dev = next(self.parameters()).device
        return self.forward_planes(planes_from_boards(x, self.width, self.height).to(dev))

    def __call__(self, state, player=1):
        """`net(state, player) -> (list[A], float)` (modules.py:109-112): single-board call."""
        state = torch.as_tensor(state) * player
        policy, value = super().__call__(state)
        return policy.tolist()[0], value.item() * player


class InferenceTower(nn.Module):
    """Frozen leaf-evaluation copy of a ResidualTower for the arena hot loop.

    BatchNorm (eval statistics) is folded into the preceding convolution, the
    weights are cast to `dtype` and activations run channels_last, so each
    block is conv(+bias)->ReLU->conv(+bias)+x->ReLU: the exact eval-mode
    function of the source tower (dropout is the identity in eval), evaluated
    in bf16.  Refresh with `load_from(tower)` after weights change.
    """

    def __init__(self, tower: ResidualTower, dtype=torch.bfloat16):
        super().__init__()
        self.dtype = dtype
        self.width, self.height, self.action_size = tower.width, tower.height, tower.action_size
        self.load_from(tower)

    @staticmethod
    def _fold(conv, bn):
        w = conv.weight.detach().double()
        b = conv.bias.detach().double() if conv.bias is not None else torch.zeros(w.shape[0], dtype=torch.float64,
                                                                                  device=w.device)
        scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
        w = w * scale.view(-1, 1, 1, 1)
        b = (b - bn.running_mean.detach().double()) * scale + bn.bias.detach().double()
        return w, b

    @torch.no_grad()
    def load_from(self, tower):
        dt = self.dtype
        cl = torch.channels_last

        def conv_pair(conv, bn):
            w, b = self._fold(conv, bn)
            return w.to(dt).contiguous(memory_format=cl), b.to(dt)

        self.stem = conv_pair(tower.conv1, tower.bn1)
        self.blocks = [(conv_pair(blk.conv1, blk.bn1), conv_pair(blk.conv2, blk.bn2)) for blk in tower.residual_blocks]
        self.pol = conv_pair(tower.conv_policy, tower.policy_bn)
        self.val = conv_pair(tower.conv_value, tower.value_bn)
        # the reference flattens NCHW (c, x, y); reorder the head matrices for NHWC (x, y, c) flatten
        ff = tower.filter_factor
        W, H = tower.width, tower.height

        def nhwc_cols(lin):
            w = lin.weight.detach()
            return w.view(w.shape[0], ff, W, H).permute(0, 2, 3, 1).reshape(w.shape[0], -1).to(dt).contiguous()

        self.lp_w, self.lp_b = nhwc_cols(tower.linear_policy), tower.linear_policy.bias.detach().to(dt)
        self.fv_w, self.fv_b = nhwc_cols(tower.fc_value), tower.fc_value.bias.detach().to(dt)
        self.lo_w, self.lo_b = tower.linear_output.weight.detach().to(dt), tower.linear_output.bias.detach().to(dt)
        return self

    @torch.no_grad()
    def forward_planes(self, x):
        x = x.to(self.dtype).contiguous(memory_format=torch.channels_last)
        (w, b) = self.stem
        x = F.relu(F.conv2d(x, w, b, padding=1))
        for (w1, b1), (w2, b2) in self.blocks:
            y = F.relu(F.conv2d(x, w1, b1, padding=1))
            x = F.relu(F.conv2d(y, w2, b2, padding=1) + x)
        p = F.relu(F.conv2d(x, self.pol[0], self.pol[1]))
        v = F.relu(F.conv2d(x, self.val[0], self.val[1]))
        # channels_last storage is already (B, x, y, c): flatten without a copy
        p = p.permute(0, 2, 3, 1).reshape(p.shape[0], -1)
        v = v.permute(0, 2, 3, 1).reshape(v.shape[0], -1)
        probs = torch.softmax(F.linear(p, self.lp_w, self.lp_b).float(), dim=1)
        v = F.relu(F.linear(v, self.fv_w, self.fv_b))
        value = torch.tanh(F.linear(v, self.lo_w, self.lo_b).float())
        return probs, value
