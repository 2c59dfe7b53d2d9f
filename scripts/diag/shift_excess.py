"""Bench-mode search shift of the fused tower (tests/test_gpu_statistical.py test_fused_tower_search_shift and the
negative controls of test_resnet_statistical_check_has_power), printed instead of asserted: for each precision and
G6 position, max |tower - fp32-evaluator| of the mean visit fractions and max excess over 4.5 SE against the
reference's own threaded samples; for the negative controls (half budget, serial search, Dirichlet alpha 0.3) the
max excess at every G6 position."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_gpu_statistical import N_RESNET_POS, _g6, _gpu_threaded, _ref_samples, _resnet_evaluator  # noqa: E402

d = _g6("resnet_single")
out = {}
for precision in ("fp16", "bf16"):
    ev = _resnet_evaluator(d, precision)
    for pi in range(N_RESNET_POS):
        pos = d["positions"][pi]
        cp, _ = _ref_samples(pos)
        fp, _, _ = _gpu_threaded(pos["opening"], 4096, d["sims"], d["thread_count"], net=_resnet_evaluator(d))
        bp, _, _ = _gpu_threaded(pos["opening"], 4096, d["sims"], d["thread_count"], net=ev)
        se = np.sqrt(cp.var(0, ddof=1) / len(cp) + bp.var(0, ddof=1) / len(bp))
        out[f"{precision}_pos{pi}"] = {"vs_fp32_max": float(np.abs(bp.mean(0) - fp.mean(0)).max()),
                                       "vs_ref_excess_max": float((np.abs(bp.mean(0) - cp.mean(0)) - 4.5 * se).max())}
    for variant in ("sims100", "serial", "alpha03"):
        ex = []
        for pi in range(N_RESNET_POS):
            pos = d["positions"][pi]
            cp, _ = _ref_samples(pos)
            sims, K, alpha = {"sims100": (100, d["thread_count"], 1.0), "serial": (d["sims"], 1, 1.0),
                              "alpha03": (d["sims"], d["thread_count"], 0.3)}[variant]
            gp, _, _ = _gpu_threaded(pos["opening"], 4096, sims, K, net=ev, alpha=alpha)
            se = np.sqrt(cp.var(0, ddof=1) / len(cp) + gp.var(0, ddof=1) / len(gp))
            ex.append(float((np.abs(gp.mean(0) - cp.mean(0)) - 4.5 * se).max()))
            if variant == "alpha03":
                ex[-1] = dict(excess=ex[-1], shift_vs_ref_max=float(np.abs(gp.mean(0) - cp.mean(0)).max()),
                              se_max=float(se.max()), ref_samples=len(cp))
        out[f"{precision}_neg_{variant}"] = {"vs_ref_excess_per_position": ex}
print(json.dumps(out, indent=1))
