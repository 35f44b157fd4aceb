"""GPU parity of the fused AutoInt head (rs_mlp_head_train + rs_partials_reduce_adam) against a
float64 torch-CPU autograd restatement of autoint:38-52 + rank/ctr/base_model.py:7-12:
  deep = MLP(x0); z = [deep | il] W3 + b3; p = clip(act3(z), 1e-6, 1); loss = mean_b sum_t CE.
Tolerances as in tests/test_gpu_parity.py: predictions / loss 1e-5 absolute, gradients
1e-4 |ref| + max(1e-4, 2e-6 max|ref|).  Ragged batches (B not a multiple of the 16-row tile),
a single deep layer and T > 1 are covered."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle
from tests._tol import assert_close, assert_grad_close, to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"
ACT = {"none": 0, "relu": 1, "sigmoid": 2}


def _act(x, a):
    return torch.relu(x) if a == "relu" else torch.sigmoid(x) if a == "sigmoid" else x


def _ref(x0, il, Ws, bs, acts, W3, b3, act3, labels):
    ps = [t.clone().requires_grad_(True) for t in [x0, il, *Ws, *bs, W3, b3]]
    x, ilr = ps[0], ps[1]
    n = len(Ws)
    Wr, br = ps[2:2 + n], ps[2 + n:2 + 2 * n]
    W3r, b3r = ps[2 + 2 * n], ps[3 + 2 * n]
    h = x
    for W, b, a in zip(Wr, br, acts):
        h = _act(h @ W + b, a)
    cat = torch.cat([h, ilr], dim=1)
    y = _act(cat @ W3r + b3r, act3)
    p = torch.clamp(y, 1e-6, 1.0)
    loss = (-labels * torch.log(p + 1e-6) - (1 - labels) * torch.log(1 - p + 1e-6)).sum(1).mean()
    loss.backward()
    return p.detach(), loss.detach(), [q.grad for q in ps]


@pytest.mark.parametrize("B,K0,S,units,acts,T,act3", [
    (1000, 416, 416, (32, 16), ("relu", "relu"), 1, "sigmoid"),   # config 2 shape, ragged B
    (4096, 416, 416, (32, 16), ("relu", "relu"), 1, "sigmoid"),
    (77, 64, 32, (64,), ("none",), 3, "sigmoid"),
    (130, 48, 24, (64, 32), ("sigmoid", "relu"), 2, "none"),
])
def test_mlp_head_matches_autograd(B, K0, S, units, acts, T, act3):
    g = torch.Generator().manual_seed(B + K0)
    f64 = torch.float64
    x0 = (torch.rand(B, K0, generator=g, dtype=f64) - 0.5)
    il = (torch.rand(B, S, generator=g, dtype=f64) - 0.5)
    dims = [K0, *units]
    Ws = [(torch.rand(dims[i], dims[i + 1], generator=g, dtype=f64) - 0.5) * 0.4 for i in range(len(units))]
    bs = [(torch.rand(dims[i + 1], generator=g, dtype=f64) - 0.5) * 0.1 for i in range(len(units))]
    C = units[-1] + S
    W3 = (torch.rand(C, T, generator=g, dtype=f64) - 0.5) * 0.2
    b3 = (torch.rand(T, generator=g, dtype=f64) - 0.5) * 0.1
    labels = (torch.rand(B, T, generator=g, dtype=f64) < 0.3).to(f64)
    # round inputs to fp32 first so both sides see the same values
    r32 = lambda t: t.float().double()
    x0, il, W3, b3 = r32(x0), r32(il), r32(W3), r32(b3)
    Ws, bs = [r32(w) for w in Ws], [r32(b) for b in bs]
    p_ref, loss_ref, grads = _ref(x0, il, Ws, bs, acts, W3, b3, act3, labels)

    d = lambda t: t.float().to(DEV).contiguous()
    N1 = units[0]
    N2 = units[1] if len(units) > 1 else 0
    lib = _lib.load()
    npar = int(lib.rs_mlp_head_param_floats(K0, N1, N2, S, T))
    nblk = int(lib.rs_mlp_head_partial_blocks(B))
    ws = torch.full((int(lib.rs_mlp_head_workspace_floats(B, K0, N1, N2, S, T)),), float("nan"),
                    device=DEV)
    assert ws.numel() == nblk * (npar + 1)
    p = torch.empty(B, T, device=DEV)
    dil = torch.empty(B, S, device=DEV)
    dx0 = torch.full((B, K0), 7.0, device=DEV)
    xd, ild = d(x0), d(il)
    Wd, bd = [d(w) for w in Ws], [d(b) for b in bs]
    W3d, b3d, lbd = d(W3), d(b3), d(labels)
    s = stream_handle()
    call("rs_mlp_head_train", s, ptr(xd), K0, ptr(ild), S, B, K0, S, N1, ACT[acts[0]], N2,
         ACT[acts[1]] if N2 else 0, T, ACT[act3], ptr(Wd[0]), ptr(bd[0]),
         ptr(Wd[1]) if N2 else None, ptr(bd[1]) if N2 else None, ptr(W3d), ptr(b3d), ptr(lbd),
         1e-6, 1.0, 1e-6, ptr(p), ptr(dil), S, ptr(dx0), K0, 0, ptr(ws), ws.numel())
    grad = torch.empty(npar, device=DEV)
    loss = torch.empty(1, device=DEV)
    _lib.partials_reduce_adam(s, [(ptr(ws), npar + 1, nblk, npar, ptr(grad), 1.0, -1),
                                  (ws.data_ptr() + 4 * npar, npar + 1, nblk, 1, ptr(loss), 1.0 / B, -1)])
    torch.cuda.synchronize()
    assert_close(to_np(p), p_ref.numpy(), 1e-5, what="p")
    assert abs(float(loss) - float(loss_ref)) <= 1e-5 * max(1.0, abs(float(loss_ref)))
    assert_grad_close(to_np(dx0), grads[0].numpy(), "dx0")
    assert_grad_close(to_np(dil), grads[1].numpy(), "dil")
    n = len(Ws)
    want = []
    for i in range(n):
        want += [grads[2 + i].reshape(-1), grads[2 + n + i].reshape(-1)]
    want += [grads[2 + 2 * n].reshape(-1), grads[3 + 2 * n].reshape(-1)]
    want = torch.cat(want).numpy()
    assert_grad_close(to_np(grad), want, "arena-order weight grads")


def test_mlp_head_dx_accumulate_and_reduce_determinism():
    B, K0, S = 513, 416, 416
    g = torch.Generator(device=DEV).manual_seed(5)
    x0 = torch.rand(B, K0, device=DEV, generator=g) - 0.5
    il = torch.rand(B, S, device=DEV, generator=g) - 0.5
    W1 = (torch.rand(K0, 32, device=DEV, generator=g) - 0.5) * 0.2
    W2 = (torch.rand(32, 16, device=DEV, generator=g) - 0.5) * 0.2
    W3 = (torch.rand(16 + S, 1, device=DEV, generator=g) - 0.5) * 0.2
    b1, b2, b3 = torch.zeros(32, device=DEV), torch.zeros(16, device=DEV), torch.zeros(1, device=DEV)
    lab = (torch.rand(B, 1, device=DEV, generator=g) < 0.5).float()
    lib = _lib.load()
    npar = int(lib.rs_mlp_head_param_floats(K0, 32, 16, S, 1))
    nblk = int(lib.rs_mlp_head_partial_blocks(B))
    ws = torch.empty(nblk * (npar + 1), device=DEV)
    dil = torch.empty(B, S, device=DEV)
    base = torch.rand(B, K0, device=DEV, generator=g)
    outs = []
    for acc in (0, 1, 1):
        dx0 = base.clone()
        call("rs_mlp_head_train", stream_handle(), ptr(x0), K0, ptr(il), S, B, K0, S, 32, 1, 16, 1,
             1, 2, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(W3), ptr(b3), ptr(lab), 1e-6, 1.0, 1e-6,
             None, ptr(dil), S, ptr(dx0), K0, acc, ptr(ws), ws.numel())
        grad = torch.empty(npar, device=DEV)
        _lib.partials_reduce_adam(stream_handle(), [(ptr(ws), npar + 1, nblk, npar, ptr(grad), 1.0, -1)])
        outs.append((dx0, grad))
    torch.cuda.synchronize()
    # accumulate adds exactly the overwrite result; two identical runs are bitwise equal
    assert torch.allclose(outs[1][0] - base, outs[0][0], atol=1e-6)
    assert torch.equal(outs[1][0], outs[2][0])
    assert torch.equal(outs[1][1], outs[2][1])


def test_partials_reduce_adam_matches_dense_adam():
    """Fused reduce + Adam == column sums then rs_dense_adam (same tf.keras Adam form), and the
    step counter advances once per launch."""
    n, rows = 3000, 37
    g = torch.Generator(device=DEV).manual_seed(9)
    part = torch.randn(rows, n + 5, device=DEV, generator=g)
    p0 = torch.randn(n, device=DEV, generator=g)
    pa, pb = p0.clone(), p0.clone()
    ma, va, mb, vb = (torch.zeros(n, device=DEV) for _ in range(4))
    sa, sb = torch.zeros(1, dtype=torch.int64, device=DEV), torch.zeros(1, dtype=torch.int64, device=DEV)
    done = torch.zeros(288, dtype=torch.int32, device=DEV)
    ga, gb = torch.empty(n, device=DEV), torch.empty(n, device=DEV)
    for _ in range(3):
        # split into two segments to exercise the segment map
        k = 1234
        _lib.partials_reduce_adam(stream_handle(), [
            (ptr(part), n + 5, rows, k, ptr(ga), 1.0, 0),
            (part.data_ptr() + 4 * k, n + 5, rows, n - k, ga.data_ptr() + 4 * k, 1.0, k)],
            pa, ma, va, sa, done, 1e-3, 0.9, 0.999, 1e-8, 0.5, True)
        gb.copy_(part[:, :n].double().sum(0).float())
        call("rs_dense_adam", stream_handle(), ptr(pb), ptr(gb), ptr(mb), ptr(vb), n, ptr(sb), 1e-3,
             0.9, 0.999, 1e-8, 0.5, 0)
    torch.cuda.synchronize()
    assert int(sa.item()) == 3 and int(done.abs().sum().item()) == 0
    assert_close(to_np(ga), part[:, :n].double().sum(0).cpu().numpy(), 1e-4, 1e-5, what="grad")
    assert_close(to_np(pa), to_np(pb), 1e-6, 1e-5, what="params")


@pytest.mark.parametrize("B,K0,S,units,acts,T,act3", [
    (1000, 416, 416, (32, 16), ("relu", "relu"), 1, "sigmoid"),   # config 2 shape, ragged B
    (4096, 416, 416, (32, 16), ("relu", "relu"), 1, "sigmoid"),
    (77, 64, 32, (64,), ("none",), 3, "sigmoid"),
    (130, 48, 24, (64, 32), ("sigmoid", "relu"), 2, "none"),
])
def test_mlp_head_deferred_w1_matches_autograd(B, K0, S, units, acts, T, act3):
    """rs_mlp_head_train_dz: dz1 rows instead of dW1 partials.  x0^T dz1 (fp64 on the host) is
    dW1; every other output / gradient as the partial-row form, against float64 autograd."""
    g = torch.Generator().manual_seed(B + K0 + 1)
    f64 = torch.float64
    r32 = lambda t: t.float().double()  # noqa: E731
    x0 = r32(torch.rand(B, K0, generator=g, dtype=f64) - 0.5)
    il = r32(torch.rand(B, S, generator=g, dtype=f64) - 0.5)
    dims = [K0, *units]
    Ws = [r32((torch.rand(dims[i], dims[i + 1], generator=g, dtype=f64) - 0.5) * 0.4) for i in range(len(units))]
    bs = [r32((torch.rand(dims[i + 1], generator=g, dtype=f64) - 0.5) * 0.1) for i in range(len(units))]
    C = units[-1] + S
    W3 = r32((torch.rand(C, T, generator=g, dtype=f64) - 0.5) * 0.2)
    b3 = r32((torch.rand(T, generator=g, dtype=f64) - 0.5) * 0.1)
    labels = (torch.rand(B, T, generator=g, dtype=f64) < 0.3).to(f64)
    p_ref, loss_ref, grads = _ref(x0, il, Ws, bs, acts, W3, b3, act3, labels)

    d = lambda t: t.float().to(DEV).contiguous()  # noqa: E731
    N1 = units[0]
    N2 = units[1] if len(units) > 1 else 0
    lib = _lib.load()
    npar = int(lib.rs_mlp_head_param_floats(K0, N1, N2, S, T))
    pn = npar - K0 * N1
    nblk = int(lib.rs_mlp_head_partial_blocks(B))
    ws = torch.full((int(lib.rs_mlp_head_dz_workspace_floats(B, K0, N1, N2, S, T)),), float("nan"),
                    device=DEV)
    assert ws.numel() == nblk * (pn + 1)
    dz1 = torch.full((B, N1 + 3), float("nan"), device=DEV)   # row stride > N1
    p = torch.empty(B, T, device=DEV)
    dil = torch.empty(B, S, device=DEV)
    dx0 = torch.full((B, K0), 7.0, device=DEV)
    xd, ild = d(x0), d(il)
    Wd, bd = [d(w) for w in Ws], [d(b) for b in bs]
    W3d, b3d, lbd = d(W3), d(b3), d(labels)
    s = stream_handle()
    call("rs_mlp_head_train_dz", s, ptr(xd), K0, ptr(ild), S, B, K0, S, N1, ACT[acts[0]], N2,
         ACT[acts[1]] if N2 else 0, T, ACT[act3], ptr(Wd[0]), ptr(bd[0]),
         ptr(Wd[1]) if N2 else None, ptr(bd[1]) if N2 else None, ptr(W3d), ptr(b3d), ptr(lbd),
         1e-6, 1.0, 1e-6, ptr(p), ptr(dil), S, ptr(dx0), K0, 0, ptr(ws), ws.numel(), ptr(dz1), N1 + 3)
    grad = torch.empty(pn, device=DEV)
    loss = torch.empty(1, device=DEV)
    _lib.partials_reduce_adam(s, [(ptr(ws), pn + 1, nblk, pn, ptr(grad), 1.0, -1),
                                  (ws.data_ptr() + 4 * pn, pn + 1, nblk, 1, ptr(loss), 1.0 / B, -1)])
    torch.cuda.synchronize()
    assert torch.isfinite(dz1[:, :N1]).all()
    assert_close(to_np(p), p_ref.numpy(), 1e-5, what="p")
    assert abs(float(loss) - float(loss_ref)) <= 1e-5 * max(1.0, abs(float(loss_ref)))
    assert_grad_close(to_np(dx0), grads[0].numpy(), "dx0")
    assert_grad_close(to_np(dil), grads[1].numpy(), "dil")
    dW1 = (x0.T @ dz1[:, :N1].double().cpu()).numpy()
    assert_grad_close(dW1, grads[2].numpy(), "dW1 = x0^T dz1")
    n = len(Ws)
    want = [grads[2 + n].reshape(-1)]
    for i in range(1, n):
        want += [grads[2 + i].reshape(-1), grads[2 + n + i].reshape(-1)]
    want += [grads[2 + 2 * n].reshape(-1), grads[3 + 2 * n].reshape(-1)]
    want = torch.cat(want).numpy()
    assert_grad_close(to_np(grad), want, "arena-order weight grads after W1")


@pytest.mark.parametrize("B,F", [(1, 26), (77, 26), (1000, 26), (2048, 26), (4099, 26), (300, 20)])
def test_il_backward_carries_deferred_weight_grad(B, F):
    """rs_il_bwd_saved_xt / rs_il_bwd_push_saved_xt (the wide kernels up to B = 1536, bwd4 above):
    the slab's rs_il_xt_splits(B) rows sum to x^T dz (fp64 reference) for an arbitrary
    [B, K0] x [B, N1] pair, and the InteractingLayer results are bitwise those of the launch
    without it."""
    E = U = 16
    H, L = 2, 3
    K0, N1 = 416, 32
    g = torch.Generator(device=DEV).manual_seed(B + F)
    lib = _lib.load()
    s = stream_handle()
    x = (torch.rand(B, F, E, device=DEV, generator=g) - 0.5)
    W = (torch.rand(E, 4 * U, device=DEV, generator=g) - 0.5) * 0.6
    bb = (torch.rand(4 * U, device=DEV, generator=g) - 0.5) * 0.2
    gm = torch.rand(U, device=DEV, generator=g) + 0.5
    bt = (torch.rand(U, device=DEV, generator=g) - 0.5) * 0.2
    dy = torch.rand(B, F * U, device=DEV, generator=g) - 0.5
    xa = torch.rand(B, K0 + 8, device=DEV, generator=g) - 0.5       # row strides > K0 / N1
    dza = torch.rand(B, N1 + 4, device=DEV, generator=g) - 0.5
    n_save = int(lib.rs_il_attn_save_floats(B, F, U, H, L))
    asave = torch.empty(n_save, device=DEV)
    ws_n = int(lib.rs_il_bwd_workspace_floats(B, E, U))
    assert lib.rs_il_bwd_xt_supported(B, F, E, U, H, ws_n) > 0
    xs = torch.empty(L - 1, B, F, U, device=DEV)
    y = torch.empty(B, F * U, device=DEV)
    wargs = (ptr(W), ptr(bb), ptr(gm), ptr(bt), 1e-14, 1, 0.0, 5)
    call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, L, *wargs, ptr(y), F * U, ptr(xs),
         ptr(asave), n_save)
    ns = int(lib.rs_il_xt_splits(B))
    out = []
    for xt in (False, True):
        for push in (False, True):
            dp = torch.empty(int(lib.rs_il_param_count(E, U)), device=DEV)
            ws = torch.empty(ws_n, device=DEV)
            dx = torch.zeros(B, F * E, device=DEV)
            table = torch.zeros(B * F, E, device=DEV)
            flag = torch.full((B * F,), -1, dtype=torch.int32, device=DEV)
            rows = torch.arange(B * F, dtype=torch.int32, device=DEV)
            slab = torch.full((ns * K0 * N1,), float("nan"), device=DEV)
            xta = (ptr(xa), K0 + 8, ptr(dza), N1 + 4, K0, N1, ptr(slab)) if xt else ()
            if push:
                call("rs_il_bwd_push_saved_xt" if xt else "rs_il_bwd_push_saved", s, ptr(x),
                     ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, *wargs, None, ptr(rows),
                     ptr(table), ptr(flag), ptr(dp), 0, ptr(ws), ws_n, ptr(asave), n_save, *xta)
            else:
                call("rs_il_bwd_saved_xt" if xt else "rs_il_bwd_saved", s, ptr(x), ptr(xs),
                     ptr(dy), F * U, B, F, E, U, H, L, *wargs, ptr(dx), 0, ptr(dp), 0, ptr(ws),
                     ws_n, ptr(asave), n_save, *xta)
            torch.cuda.synchronize()
            out.append((dp.clone(), (table if push else dx).clone()))
            if xt:
                ref = xa[:, :K0].double().T @ dza[:, :N1].double()
                got = slab.view(ns, K0, N1).double().sum(0)
                assert_close(got.cpu().numpy(), ref.cpu().numpy(), 1e-4, 1e-5,
                             what=f"x^T dz slab rows (push={push})")
    for k in (0, 1):
        assert torch.equal(out[k][0], out[k + 2][0]) and torch.equal(out[k][1], out[k + 2][1])
