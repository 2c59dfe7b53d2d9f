"""BatchNorm over channels-last rows [N, C] on the GPU in fp16 (train mode, fp32 weights), forward and
backward, against the fp32 reference: MIOpen with a 2-D input (per-activation mode), MIOpen with
[N, C, 1, 1] (spatial mode), and PyTorch's own kernels with a 2-D input (cudnn/MIOpen disabled);
max errors, NaNs and the time per forward+backward."""
import time

import torch
import torch.nn.functional as F

torch.manual_seed(0)
N, C = 64 * 42, 128
y0 = (torch.randn(N, C, device="cuda") * 3 + 1).half()
gy = torch.randn(N, C, device="cuda").half()
w0 = torch.rand(C, device="cuda") + 0.5
b0 = torch.randn(C, device="cuda")


def run(f, y, w, b, lib=True, half=True):
    y = y.detach().clone().requires_grad_(True)
    w = w.detach().clone().requires_grad_(True)
    b = b.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    with torch.backends.cudnn.flags(enabled=lib):
        out = F.batch_norm(f(y), rm, rv, w, b, True, 0.1, 1e-5).reshape(N, C)
        out.backward(gy if half else gy.float())
    return out.float(), y.grad.float(), w.grad, b.grad, rm, rv


ref = run(lambda t: t, y0.float(), w0, b0, lib=False, half=False)
for name, f, lib in (("miopen_2d", lambda t: t, True), ("miopen_n_c_1_1", lambda t: t.view(N, C, 1, 1), True),
                     ("native_2d", lambda t: t, False)):
    got = run(f, y0, w0, b0, lib=lib)
    errs = [float((a - r).abs().max()) for a, r in zip(got, ref)]
    nan = [bool(torch.isnan(a).any()) for a in got]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        run(f, y0, w0, b0, lib=lib)
    torch.cuda.synchronize()
    print(name, "max err out/dy/dw/db/rm/rv", [round(e, 5) for e in errs], "nan", nan,
          "us per fwd+bwd (incl. clones)", round((time.perf_counter() - t0) / 50 * 1e6, 1), flush=True)
