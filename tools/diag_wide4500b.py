"""Diagnostic: the wide IL pair's dx at B = 4500 vs the float64 twin, on the full batch and on
sub-batches containing sample 2272 (which differed), to tell a data- from a position-dependent
fault."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import torch_ref as tr  # noqa: E402
from test_gpu_il_wide import _params, _run  # noqa: E402

B, F, L = 4500, 26, 3
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(B * 7 + F * 3 + L)
x = torch.rand(B, F, 16, device=dev, generator=g) - 0.5
prm = _params(g)
dy = torch.randn(B, F * 16, device=dev, generator=g)
base = torch.randn(B, F * 16, device=dev, generator=g)
rows = torch.randint(-1, 300, (B * F,), device=dev, dtype=torch.int32, generator=g)
xr = x.detach().double().cpu().requires_grad_(True)
W, b, gm, bt = (p.detach().double().cpu().requires_grad_(True) for p in prm)
tr.interacting_layer(xr, W, b, gm, bt, L, 2, True).backward(dy.double().cpu().view(B, F, 16))
ref = xr.grad.numpy().reshape(B, F * 16) + base.double().cpu().numpy()
np.set_printoptions(precision=4, suppress=True, linewidth=200)
for lo, hi in ((0, 4500), (2272, 2273), (0, 2500), (1000, 4500), (2000, 4500), (2200, 2300)):
    n = hi - lo
    for var in ("wide", "wave"):
        out = _run(var, n, F, L, 0.0, False, x[lo:hi].contiguous(), prm, dy[lo:hi].contiguous(),
                   base[lo:hi].contiguous(), rows[lo * F:hi * F].contiguous())
        dx = out[2].double().cpu().numpy()
        err = np.abs(dx - ref[lo:hi]).max(axis=1)
        bad = np.nonzero(err > 1e-3)[0] + lo
        print(f"[{lo},{hi}) {var}: bad {len(bad)} {bad[:10].tolist()} max {err.max():.3e}", flush=True)
        if var == "wide" and len(bad):
            k = bad[0] - lo
            e = np.abs(dx[k] - ref[bad[0]]).reshape(F, 16)
            print("  per-field max err", e.max(axis=1), flush=True)
