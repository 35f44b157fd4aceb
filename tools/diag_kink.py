"""Verdict r04 item 1: is the wide IL backward's dx disagreement at sample 2272 (B = 4500, F = 26,
L = 3, test_gpu_il_wide.py's seeded inputs) a ReLU kink or a kernel bug?

1. runs the wide and the one-wave kernel pairs on the test's inputs (GPU);
2. float64 twin (InteractingLayer.py:37-61 op for op) with every projection ReLU's pre-activation
   z recorded, and its margin |z| / (sum_e |x_e W_ec| + |b_c|) -- how far z lies from the kink in
   units of its own magnitude (fp32 rounding of z is ~1e-7 of that, plus the propagated
   difference of the fp32 inputs of layers 1, 2);
3. for the smallest-margin ReLUs of the disagreeing sample: the float64 dx with THAT ONE ReLU's
   derivative flipped, compared with the wide and the one-wave kernels' dx.
(relu(O + R) needs no check: O and R are post-ReLU, so O + R >= 0 and is 0 only when both are.)
Output: profiles/r05/kink/ (committed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import torch_ref as tr  # noqa: E402
from test_gpu_il_wide import _params, _run  # noqa: E402

B, F, L, H, U = 4500, 26, 3, 2, 16


def twin(x, W, b, gm, bt, flips=()):
    """float64 IL; flips: (it, c, f, u) ReLU derivatives to flip (c: 0..3 = Q, K, V, R).
    Returns (y, [per-iteration (z, scale)])."""
    out = x
    rec = []
    for it in range(L):
        z = torch.einsum("bfe,ec->bfc", out, W) + b                          # [B, F, 4U]
        scale = torch.einsum("bfe,ec->bfc", out.abs(), W.abs()) + b.abs()
        rec.append((z.detach(), scale.detach()))
        keep = (z > 0).double()
        for (fi, c, f, u) in flips:
            if fi == it:
                keep = keep.clone()
                keep[0, f, c * U + u] = 1.0 - keep[0, f, c * U + u]
        pr = z * keep                       # relu with the (possibly flipped) derivative mask
        q, k, v, r = (pr[..., j * U:(j + 1) * U] for j in range(4))
        o = torch.zeros_like(q)
        dh = U // H
        for h in range(H):
            sl = slice(dh * h, dh * h + dh)
            w = torch.softmax(q[..., sl] @ k[..., sl].transpose(1, 2) / dh ** 0.5, dim=-1)
            o[..., sl] = w @ v[..., sl]
        out = tr.layer_norm(torch.relu(o + r), gm, bt, 1e-14)
    return out, rec


def main():
    out_dir = os.path.join(ROOT, "profiles", "r05", "kink")
    os.makedirs(out_dir, exist_ok=True)
    lines = []

    def log(s):
        print(s, flush=True)
        lines.append(s)

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(B * 7 + F * 3 + L)
    x = torch.rand(B, F, 16, device=dev, generator=g) - 0.5
    prm = _params(g)
    dy = torch.randn(B, F * 16, device=dev, generator=g)
    base = torch.randn(B, F * 16, device=dev, generator=g)
    rows = torch.randint(-1, 300, (B * F,), device=dev, dtype=torch.int32, generator=g)
    got = {}
    for var in ("wide", "wave"):
        res = _run(var, B, F, L, 0.0, False, x, prm, dy, base, rows)
        got[var] = (res[2].double().cpu().numpy() - base.double().cpu().numpy()).reshape(B, F, 16)
    W, b, gm, bt = (p.detach().double().cpu() for p in prm)
    xd = x.detach().double().cpu().requires_grad_(True)
    dyd = dy.double().cpu().view(B, F, 16)
    y, rec = twin(xd, W, b, gm, bt)
    y.backward(dyd)
    ref = xd.grad.numpy()
    # per-sample minimal margin over every projection ReLU of every iteration
    marg = np.stack([(z.abs() / s).reshape(B, -1).min(dim=1).values.numpy() for z, s in rec], 1).min(1)
    amax = np.abs(ref).max()
    for var in ("wide", "wave"):
        err = np.abs(got[var] - ref).reshape(B, -1).max(1)
        bad = np.nonzero(err > 1e-4 + 2e-6 * amax + 1e-4 * np.abs(ref).reshape(B, -1).max(1))[0]
        log(f"{var}: samples outside the gradient tolerance: {bad.tolist()[:20]}  max err {err.max():.3e}"
            f"  (max err over the others {np.delete(err, bad).max():.3e})")
    order = np.argsort(marg)
    log("smallest per-sample ReLU margins |z|/sum|terms| (sample: margin):  " +
        "  ".join(f"{int(s)}: {marg[s]:.2e}" for s in order[:12]))
    log(f"margin quantiles: 1e-3 {np.quantile(marg, 1e-3):.2e}  1e-2 {np.quantile(marg, 1e-2):.2e}  "
        f"median {np.median(marg):.2e}")
    s = 2272
    cand = []
    for it, (z, sc) in enumerate(rec):
        m = (z[s].abs() / sc[s]).numpy()                     # [F, 4U]
        for flat in np.argsort(m, axis=None)[:6]:
            f, cu = np.unravel_index(flat, m.shape)
            cand.append((float(m[f, cu]), it, int(cu) // U, int(f), int(cu) % U, float(z[s, f, cu])))
    cand.sort()
    xs = xd.detach()[s:s + 1].clone()
    ys = dyd[s:s + 1]
    gw, gv, rs_ = got["wide"][s], got["wave"][s], ref[s]
    log(f"sample {s}: |dx_wide - dx64| max {np.abs(gw - rs_).max():.3e}, "
        f"|dx_wave - dx64| max {np.abs(gv - rs_).max():.3e}")
    log("candidate ReLUs of sample 2272, smallest margin first; dx64 with that ReLU's derivative "
        "flipped vs each kernel:")
    for mg, it, c, f, u, zval in cand[:12]:
        xr = xs.clone().requires_grad_(True)
        yf, _ = twin(xr, W, b, gm, bt, flips=[(it, c, f, u)])
        yf.backward(ys)
        dxf = xr.grad.numpy()[0]
        log(f"  it {it} {'QKVR'[c]} field {f:2d} unit {u:2d}: z {zval:+.3e} margin {mg:.2e} | "
            f"flipped-vs-wide {np.abs(dxf - gw).max():.3e}  flipped-vs-wave {np.abs(dxf - gv).max():.3e}"
            f"  flipped-vs-unflipped {np.abs(dxf - rs_).max():.3e}")
    with open(os.path.join(out_dir, "diag_kink.txt"), "w") as fh:
        fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
