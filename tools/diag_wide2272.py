"""Diagnostic: conditioning of sample 2272 of the B = 4500 wide-IL test batch -- the float64 LN
variance per (layer, field) and the float64 dx's change under a 1e-7 relative perturbation of x."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from oracle import torch_ref as tr  # noqa: E402
from test_gpu_il_wide import _params  # noqa: E402

B, F, L = 4500, 26, 3
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(B * 7 + F * 3 + L)
x = torch.rand(B, F, 16, device=dev, generator=g) - 0.5
prm = _params(g)
dy = torch.randn(B, F * 16, device=dev, generator=g)
s = 2272
W, b, gm, bt = (p.detach().double().cpu() for p in prm)
x1 = x[s:s + 1].double().cpu()
d1 = dy[s:s + 1].double().cpu().view(1, F, 16)
# per-layer LN input variance
out = x1
for it in range(L):
    U = 16
    pr = torch.relu(out @ W + b)
    q, k, v, r = (pr[..., j * U:(j + 1) * U] for j in range(4))
    o = torch.zeros_like(q)
    for h in range(2):
        sl = slice(8 * h, 8 * h + 8)
        w = torch.softmax(q[..., sl] @ k[..., sl].transpose(1, 2) / 8 ** 0.5, dim=-1)
        o[..., sl] = w @ v[..., sl]
    z = torch.relu(o + r)
    var = z.var(dim=-1, unbiased=False)[0]
    print(f"layer {it}: min var {var.min():.3e} at field {int(var.argmin())}; field 18 var {var[18]:.3e}; "
          f"field 18 z {z[0, 18].numpy()}", flush=True)
    out = tr.layer_norm(z, gm, bt, 1e-14)
for eps in (0.0, 1e-7, -1e-7, 1e-6):
    xr = (x1 * (1 + eps * torch.sign(torch.sin(torch.arange(x1.numel(), dtype=torch.float64).view_as(x1) * 7.1)))
          ).requires_grad_(True)
    tr.interacting_layer(xr, W, b, gm, bt, L, 2, True).backward(d1)
    if eps == 0.0:
        base = xr.grad.clone()
    print(f"perturb {eps:+.0e}: max |dx - dx0| = {(xr.grad - base).abs().max():.3e}, "
          f"field 18 max |dx| {xr.grad[0, 18].abs().max():.3e}", flush=True)
