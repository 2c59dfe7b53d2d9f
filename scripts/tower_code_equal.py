"""Bit-equality of a timing alternative (SPMCTS_TOWER_CG) with the default trunk: run once per code
(the switch is read once per process) writing the host-path outputs, then compare the files.
  python scripts/tower_code_equal.py dump OUT.npz [FILTER_FACTOR [bf16|fp16]]   |   python scripts/tower_code_equal.py cmp A.npz B.npz"""
import sys

import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(out, ff=32, dtype="bf16"):
    import torch

    from self_play_reinforcement_learning_amd.evaluator import HipTowerEvaluator
    from self_play_reinforcement_learning_amd.modules import ResidualTower, planes_from_boards

    res = {}
    for blocks in (2, 20):
        torch.manual_seed(0)
        net = ResidualTower(7, 6, 7, num_blocks=blocks, filter_factor=ff)
        with torch.no_grad():
            for m in net.modules():
                if isinstance(m, torch.nn.BatchNorm2d):
                    m.running_mean.uniform_(-0.2, 0.2)
                    m.running_var.uniform_(0.5, 2.0)
        net = net.cuda().eval()
        b = np.random.default_rng(1).choice([-1, 0, 1], size=(4000, 7, 6), p=[0.3, 0.4, 0.3])
        x = planes_from_boards(torch.as_tensor(b), 7, 6).cuda()
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ev = HipTowerEvaluator(net, dtype={"bf16": torch.bfloat16, "fp16": torch.float16}[dtype])
        p, v = ev(x)
        res[f"p{blocks}"] = p.float().cpu().numpy()
        res[f"v{blocks}"] = v.float().cpu().numpy()
        # the device-count path (k_tower_dyn) on a ragged batch: whole rounds + tail tiles
        n = 3001
        cnt = torch.tensor([n], dtype=torch.int32, device="cuda")
        pd, vd = ev.forward_dev(x, cnt, 4000)
        res[f"pd{blocks}"] = pd[:n].float().cpu().numpy()
        res[f"vd{blocks}"] = vd[:n].float().cpu().numpy()
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k])]
    print({"equal": not bad, "differ": bad,
           "max_abs": {k: float(np.abs(A[k] - B[k]).max()) for k in A.files}})
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 32, sys.argv[4] if len(sys.argv) > 4 else "bf16")
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
