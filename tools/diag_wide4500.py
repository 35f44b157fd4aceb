"""Diagnostic: which samples' dx differ between the wide / wave IL pairs at B = 4500 (past the
wide forward's grid), each against the float64 autograd twin.  RS_IL_WIDE_FWD_GRID varies the
forward grid."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import torch_ref as tr  # noqa: E402
from test_gpu_il_wide import _params, _run  # noqa: E402

B, F, L = int(os.environ.get("DIAG_B", "4500")), 26, 3
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
ref = xr.grad.numpy().reshape(B, F * 16) + base.double().cpu().numpy()  # dx accumulates onto base
for var in ("wave", "wide"):
    out = _run(var, B, F, L, 0.0, False, x, prm, dy, base, rows)
    dx = out[2].double().cpu().numpy()
    err = np.abs(dx - ref).max(axis=1)
    bad = np.nonzero(err > 1e-3)[0]
    print(var, "fwd grid", os.environ.get("RS_IL_WIDE_FWD_GRID", "default"), "bad samples", len(bad),
          bad[:20].tolist(), bad[-5:].tolist() if len(bad) else [], "max", float(err.max()), flush=True)
