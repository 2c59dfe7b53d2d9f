"""BatchNorm over channels-last rows on the GPU under fp16 autocast: [N, C] (MIOpen per-activation
mode) vs [N, C, 1, 1] (spatial mode) vs the fp32 reference, train mode; prints max errors / NaNs and
the time per call."""
import time

import torch
import torch.nn.functional as F

torch.manual_seed(0)
N, C = 64 * 42, 128
y = (torch.randn(N, C, device="cuda") * 3 + 1).half()
w = torch.rand(C, device="cuda") + 0.5
b = torch.randn(C, device="cuda")
ref = F.batch_norm(y.float(), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"), w, b, True, 0.1, 1e-5)
for name, f in (("2d", lambda t: t), ("4d_n_c_1_1", lambda t: t.view(N, C, 1, 1))):
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    with torch.autocast("cuda", dtype=torch.float16):
        out = F.batch_norm(f(y), rm, rv, w, b, True, 0.1, 1e-5).view(N, C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        F.batch_norm(f(y), rm, rv, w, b, True, 0.1, 1e-5)
    torch.cuda.synchronize()
    print(name, out.dtype, "nan", bool(out.isnan().any()), "max err", float((out.float() - ref).abs().max()),
          "rm err", float((rm - 0.1 * y.float().mean(0)).abs().max()), "us/call", (time.perf_counter() - t0) / 200 * 1e6)
