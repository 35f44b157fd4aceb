"""H3 InteractingLayer, one 4-wave workgroup per sample (il_wide.hpp; rs_il_set_variant 2) for
the AutoInt shape family (E = U = 16, H = 2, F <= 32; InteractingLayer.py:37-61).

Checked against the float64 oracle (forward 1e-5, gradients at the gradient tolerance) and
against the one-wave-per-sample kernels (variant 1) on the same inputs: forward, saved-path
backward with and without the fused sparse push, dropout, small / padded F, a single sample,
and batches larger than the kernels' grids (the persistent sample loops)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from oracle import torch_ref as tr

from _tol import assert_close, assert_grad_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
E = U = 16
H = 2


def _np(t):
    return t.detach().double().cpu().numpy()


def _params(g):
    W = (torch.rand(E, 4 * U, device=DEV, generator=g) - 0.5) * 0.6
    b = (torch.rand(4 * U, device=DEV, generator=g) - 0.5) * 0.2
    gm = torch.rand(U, device=DEV, generator=g) + 0.5
    bt = (torch.rand(U, device=DEV, generator=g) - 0.5) * 0.2
    return W, b, gm, bt


def _run(variant, B, F, L, drop, push, x, prm, dy, base, rows):
    """forward (saved) + backward (saved / push) under one kernel variant"""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import call, ptr, stream_handle
    lib = _lib.load()
    W, b, gm, bt = prm
    s = stream_handle()
    with _lib.il_variant(variant):
        n_save = int(lib.rs_il_attn_save_floats(B, F, U, H, L))
        asave = torch.full((n_save,), float("nan"), device=DEV)
        ws_n = int(lib.rs_il_bwd_workspace_floats(B, E, U))
        nb = int(lib.rs_il_bwd_saved_partial_blocks(B, F, E, U, H, ws_n))
        npar = int(lib.rs_il_param_count(E, U))
        y = torch.empty(B, F * U, device=DEV)
        xs = torch.empty(max(L - 1, 1), B, F, U, device=DEV)
        xsp = ptr(xs) if L > 1 else None
        wargs = (ptr(W), ptr(b), ptr(gm), ptr(bt), 1e-14, 1, drop, 77)
        call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, L, *wargs, ptr(y), F * U, xsp,
             ptr(asave), n_save)
        dp = torch.empty(npar, device=DEV)
        ws = torch.full((ws_n,), float("nan"), device=DEV)
        dx = base.clone()
        table = torch.zeros(300, E, device=DEV)
        flag = torch.full((300,), -1, dtype=torch.int32, device=DEV)
        if push:
            call("rs_il_bwd_push_saved", s, ptr(x), xsp, ptr(dy), F * U, B, F, E, U, H, L, *wargs,
                 ptr(base), ptr(rows), ptr(table), ptr(flag), ptr(dp), 0, ptr(ws), ws_n,
                 ptr(asave), n_save)
        else:
            call("rs_il_bwd_saved", s, ptr(x), xsp, ptr(dy), F * U, B, F, E, U, H, L, *wargs,
                 ptr(dx), 1, ptr(dp), 0, ptr(ws), ws_n, ptr(asave), n_save)
        torch.cuda.synchronize()
        assert torch.isfinite(asave).all()
        # the per-block partial rows the backward leaves sum to the reduced parameters
        part = ws[:nb * npar].view(nb, npar)
        assert torch.isfinite(part).all()
        assert_grad_close(_np(part.double().sum(0)), _np(dp), what=f"{variant} partial rows")
    return y, xs, (table if push else dx), dp, flag


CASES = [  # (B, F, L, drop)
    (67, 26, 3, 0.0),      # config 2 (exact-F instantiation)
    (1, 26, 3, 0.0),       # one sample: one workgroup
    (2500, 26, 3, 0.0),    # more samples than the backward's grid (persistent loop)
    # more samples than the forward's grid too, at few fields and one layer: a batch has B F 64 L
    # ReLU inputs and about one in 1e7 lies within fp32 rounding of the kink, where the float64
    # dx itself jumps (B = 4500, F = 26, L = 3: sample 2272's dx moves by 1.6 under a 1e-7 relative
    # change of x, tools/diag_wide2272.py) -- two fp32 kernels may then land on either side
    (4200, 8, 1, 0.0),
    (40, 20, 2, 0.0),      # padded F (FMAX 32)
    (9, 31, 3, 0.1),       # dropout, padded
    (13, 4, 1, 0.0),       # fewer fields than key quarters + the dx-exchange buffer floor
    (30, 26, 1, 0.2),      # dropout, exact
]


@pytest.mark.parametrize("B,F,L,drop", CASES)
@pytest.mark.parametrize("push", [False, True])
def test_il_wide_matches_wave_variant(B, F, L, drop, push):
    g = torch.Generator(device=DEV).manual_seed(B * 7 + F * 3 + L)
    x = torch.rand(B, F, E, device=DEV, generator=g) - 0.5
    prm = _params(g)
    dy = torch.randn(B, F * U, device=DEV, generator=g)
    base = torch.randn(B, F * E, device=DEV, generator=g)
    rows = torch.randint(-1, 300, (B * F,), device=DEV, dtype=torch.int32, generator=g)
    wave = _run("wave", B, F, L, drop, push, x, prm, dy, base, rows)
    wide = _run("wide", B, F, L, drop, push, x, prm, dy, base, rows)
    assert_close(_np(wide[0]), _np(wave[0]), 1e-5, what="y")
    if L > 1:
        assert_close(_np(wide[1]), _np(wave[1]), 1e-5, what="xsave")
    assert_grad_close(_np(wide[2]), _np(wave[2]), what="pushed rows" if push else "dx")
    assert_grad_close(_np(wide[3]), _np(wave[3]), what="dparams")
    assert torch.equal(wide[4], wave[4])  # the same rows scan-marked


@pytest.mark.parametrize("B,F,L,drop", [(67, 26, 3, 0.0), (9, 31, 2, 0.1)])
def test_il_wide_matches_oracle(B, F, L, drop):
    """The wide pair against the float64 oracle / its autograd twin (dropout through the shared
    counter-based mask)."""
    from recommendsystem_amd.layers import InteractingLayer
    from recommendsystem_amd import _lib
    rng = np.random.default_rng(B + F)
    x = rng.uniform(-0.5, 0.5, size=(B, F, E)).astype(np.float32)
    dy = rng.normal(size=(B, F, U)).astype(np.float32)
    il = InteractingLayer(L, U, H, use_dropout=drop > 0, dropout_rate=drop, seed=8, device=DEV)
    il.build((B, F, E), device=DEV)
    il.train()
    gen = torch.Generator(device=DEV).manual_seed(9)
    with torch.no_grad():
        il.bias.uniform_(-0.1, 0.1, generator=gen)
        il.gamma.uniform_(0.5, 1.5, generator=gen)
        il.beta.uniform_(-0.2, 0.2, generator=gen)
    seed = (il.seed * 1000003 + il._calls) & 0xFFFFFFFFFFFFFFFF
    xd = torch.from_numpy(x).to(DEV).requires_grad_(True)
    with _lib.il_variant("wide"):
        y = il(xd)
        y.backward(torch.from_numpy(dy).to(DEV))
        torch.cuda.synchronize()
    prm = [_np(p) for p in (il.kernel, il.bias, il.gamma, il.beta)]
    ref = npo.interacting_layer(x.astype(np.float64), *prm, L, H, True, drop_rate=drop, seed=seed)
    assert_close(_np(y), ref, 1e-5, what="wide IL fwd vs oracle")
    W, b, gm, bt = (torch.from_numpy(a).requires_grad_(True) for a in prm)
    xr = torch.from_numpy(x).double().requires_grad_(True)
    tr.interacting_layer(xr, W, b, gm, bt, L, H, True, drop_rate=drop, seed=seed).backward(
        torch.from_numpy(dy).double())
    assert_grad_close(_np(xd.grad), xr.grad.numpy(), what="dx")
    assert_grad_close(_np(il.kernel.grad), W.grad.numpy(), what="dW")
    assert_grad_close(_np(il.bias.grad), b.grad.numpy(), what="db")
    assert_grad_close(_np(il.gamma.grad), gm.grad.numpy(), what="dgamma")
    assert_grad_close(_np(il.beta.grad), bt.grad.numpy(), what="dbeta")


def test_il_variant_switch():
    from recommendsystem_amd import _lib
    lib = _lib.load()
    assert lib.rs_il_get_variant() in (0, 1, 2)
    with _lib.il_variant("wave"):
        assert lib.rs_il_get_variant() == 1
    assert lib.rs_il_set_variant(7) == -1
