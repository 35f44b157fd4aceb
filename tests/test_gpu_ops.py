"""torch.library custom ops (recommendsystem_amd/ops.py, torch.ops.ctr.*): torch.library.opcheck
(schema, fake/meta kernels, autograd registration, AOTAutograd dispatch) on each op, parity of
the op path with the layer path, and a torch.compile(backend="aot_eager") trace of a model that
routes its layers through the ops."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from _tol import assert_close, assert_grad_close, to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _ops():
    from recommendsystem_amd import ops  # noqa: F401 (registers torch.ops.ctr)
    yield
    ops.use_custom_ops(False)


def _il_args(B=6, F=26, E=16, U=16, L=3, H=2, drop=0.0, grad=True):
    g = torch.Generator(device=DEV).manual_seed(0)
    x = (torch.rand(B, F, E, device=DEV, generator=g) - 0.5).requires_grad_(grad)
    W = ((torch.rand(E, 4 * U, device=DEV, generator=g) - 0.5) * 0.5).requires_grad_(grad)
    b = ((torch.rand(4 * U, device=DEV, generator=g) - 0.5) * 0.1).requires_grad_(grad)
    gm = (1 + (torch.rand(U, device=DEV, generator=g) - 0.5) * 0.1).requires_grad_(grad)
    bt = ((torch.rand(U, device=DEV, generator=g) - 0.5) * 0.1).requires_grad_(grad)
    return (x, W, b, gm, bt, L, H, True, 1e-14, drop, 12345)


@pytest.mark.parametrize("drop", [0.0, 0.2])
def test_opcheck_interacting(drop):
    torch.library.opcheck(torch.ops.ctr.interacting_fwd.default, _il_args(drop=drop))


def test_opcheck_dense_and_din_and_lookup():
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.rand(33, 40, device=DEV, generator=g).requires_grad_(True)
    W = (torch.rand(40, 24, device=DEV, generator=g) - 0.5).requires_grad_(True)
    b = (torch.rand(24, device=DEV, generator=g) - 0.5).requires_grad_(True)
    for act in (0, 1, 2):
        torch.library.opcheck(torch.ops.ctr.dense.default, (x, W, b, act))
    B, T, H = 5, 12, 16
    q = torch.rand(B, H, device=DEV, generator=g).requires_grad_(True)
    k = torch.rand(B, T, H, device=DEV, generator=g).requires_grad_(True)
    v = torch.rand(B, T, H, device=DEV, generator=g).requires_grad_(True)
    lens = torch.tensor([12, 3, 7, 12, 1], dtype=torch.int32, device=DEV)
    W1 = (torch.rand(3 * H, 16, device=DEV, generator=g) - 0.5).requires_grad_(True)
    b1 = torch.zeros(16, device=DEV).requires_grad_(True)
    W2 = (torch.rand(16, 1, device=DEV, generator=g) - 0.5).requires_grad_(True)
    b2 = torch.zeros(1, device=DEV).requires_grad_(True)
    torch.library.opcheck(torch.ops.ctr.din_pool.default, (q, k, v, lens, None, W1, b1, W2, b2, 0))
    W1s = (torch.rand(4 * H, 16, device=DEV, generator=g) - 0.5).requires_grad_(True)
    mask = torch.rand(B, T, device=DEV, generator=g) < 0.7
    torch.library.opcheck(torch.ops.ctr.din_pool.default, (q, k, k, None, mask, W1s, b1, W2, b2, 1))
    table = torch.rand(1000, 16, device=DEV)
    ids = torch.randint(0, 5000, (7, 4), device=DEV)
    rb = torch.tensor([0, 250, 500, 750], device=DEV)
    bk = torch.full((4,), 250, device=DEV, dtype=torch.int64)
    torch.library.opcheck(torch.ops.ctr.embedding_lookup.default, (ids, None, rb, bk, 0, 1, table))


def test_op_path_matches_layer_path():
    from recommendsystem_amd import ops
    from recommendsystem_amd.layers import InteractingLayer
    il = InteractingLayer(3, 16, 2, use_res=True, seed=5, device=DEV)
    x = (torch.rand(9, 26, 16, device=DEV) - 0.5).requires_grad_(True)
    y0 = il(x)
    y0.sum().backward()
    gx0, gW0 = x.grad.clone(), il.kernel.grad.clone()
    x.grad = None
    il.kernel.grad.zero_()
    ops.use_custom_ops(True)
    y1 = il(x)
    y1.sum().backward()
    assert torch.equal(y0, y1)
    assert torch.equal(gx0, x.grad)
    assert torch.equal(gW0, il.kernel.grad)


def test_compile_aot_eager_traces_the_ops():
    from recommendsystem_amd import ops
    from recommendsystem_amd.layers import Dense, InteractingLayer
    ops.use_custom_ops(True)
    il = InteractingLayer(3, 16, 2, use_res=True, seed=7, device=DEV)
    il.build((1, 26, 16), device=DEV)
    head = Dense(1, "sigmoid", seed=8, device=DEV)
    head.build((1, 26 * 16), device=DEV)

    def f(x):
        return head(il(x).reshape(x.shape[0], -1))

    x = (torch.rand(8, 26, 16, device=DEV) - 0.5)
    y_eager = f(x)
    cf = torch.compile(f, backend="aot_eager", fullgraph=True)
    il._calls = 0
    y_c = cf(x)
    assert_close(to_np(y_c), to_np(y_eager), 1e-6, what="compiled vs eager")
    xr = x.clone().requires_grad_(True)
    cf(xr).sum().backward()
    assert xr.grad is not None and torch.isfinite(xr.grad).all()


@pytest.mark.parametrize("M,K,N,act,acc", [
    (2048, 64, 32, 1, 0),     # 4 tiles -> split-K, reduced inside the GEMM launch
    (2048, 200, 48, 2, 1),    # ragged tiles, sigmoid Z operand, accumulate
    (4099, 96, 64, 0, 0),     # ragged M (the last split short)
    (300, 512, 256, 1, 0),    # short M: three splits
])
def test_dense_bwd_weight_split_k(M, K, N, act, acc):
    """rs_dense_bwd_weight: dW = X^T dZ, db = colsum dZ (dZ = dY * act'(Y)) against float64, for
    shapes whose plan splits the reduction (the last split of each tile sums the partials in split
    order inside the launch); two launches are bitwise equal."""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import call, ptr, stream_handle
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    X = torch.rand(M, K, device="cuda", generator=g) - 0.5
    dY = torch.rand(M, N, device="cuda", generator=g) - 0.5
    Y = torch.rand(M, N, device="cuda", generator=g) - 0.3   # relu mask ~30 % off
    if act == 2:
        Y = torch.rand(M, N, device="cuda", generator=g)
    lib = _lib.load()
    ws_n = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
    outs = []
    for _ in range(2):
        ws = torch.full((max(ws_n, 1),), float("nan"), device="cuda")
        dW = torch.full((K, N), 0.25, device="cuda")
        db = torch.full((N,), 0.5, device="cuda")
        call("rs_dense_bwd_weight", stream_handle(), ptr(X), K, ptr(dY), N, ptr(Y), N, act, M, K,
             N, ptr(dW), ptr(db), acc, ptr(ws), ws_n)
        torch.cuda.synchronize()
        outs.append((dW.clone(), db.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    Yd, dYd = Y.double(), dY.double()
    dZ = dYd * (Yd > 0) if act == 1 else dYd * Yd * (1 - Yd) if act == 2 else dYd
    rW = X.double().T @ dZ + (0.25 if acc else 0.0)
    rb = dZ.sum(0) + (0.5 if acc else 0.0)
    assert_close(to_np(outs[0][0]), rW.cpu().numpy(), 1e-4, 1e-5, what="dW")
    assert_close(to_np(outs[0][1]), rb.cpu().numpy(), 1e-4, 1e-5, what="db")


@pytest.mark.parametrize("M,K,N,act", [
    (2048, 1712, 960, 1),     # config-5 first layer: 32x32-MFMA blocks, 128 x 64
    (4099, 1616, 273, 0),     # config-3 trunk, ragged M / N, unaligned rows (scalar loads)
    (1000, 1840, 400, 2),     # ragged M, sigmoid Z operand
    (600, 1000, 700, 1),      # ragged everywhere, weight gradient split over M
])
def test_dense_large_gemm_blocks(M, K, N, act):
    """The large-GEMM blocks (v_mfma_f32_32x32x2_f32, >= 2^28 multiply-adds): forward with bias +
    activation into a strided output, data gradient accumulated into a strided dX, weight gradient
    (+ column sums, split or not) -- each against float64."""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import call, ptr, stream_handle
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    s = stream_handle()
    ldx = K + 8
    Xb = torch.rand(M, ldx, device="cuda", generator=g) - 0.5
    X = Xb[:, :K]
    W = (torch.rand(K, N, device="cuda", generator=g) - 0.5) * 0.1
    b = torch.rand(N, device="cuda", generator=g) - 0.5
    ldy = N + 4
    Yb = torch.full((M, ldy), float("nan"), device="cuda")
    call("rs_dense_fwd", s, ptr(Xb), M, K, ldx, ptr(W), ptr(b), N, act, ptr(Yb), ldy)
    torch.cuda.synchronize()
    Y = Yb[:, :N]
    Xd, Wd = X.double(), W.double()
    z = Xd @ Wd + b.double()
    ry = torch.relu(z) if act == 1 else torch.sigmoid(z) if act == 2 else z
    tol = 1e-7 * K * 0.25 * 8
    assert_close(to_np(Y), ry.cpu().numpy(), tol, 1e-5, what="fwd")
    dY = torch.rand(M, N, device="cuda", generator=g) - 0.5
    Yc = Y.contiguous()
    Yd = Yc.double()
    dZ = dY.double() * (Yd > 0) if act == 1 else dY.double() * Yd * (1 - Yd) if act == 2 else dY.double()
    dXb = torch.full((M, ldx), 0.25, device="cuda")
    call("rs_dense_bwd_data", s, ptr(dY), N, ptr(Yc), N, act, ptr(W), M, K, N, ptr(dXb), ldx, 1)
    lib = _lib.load()
    ws_n = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
    ws = torch.full((max(ws_n, 1),), float("nan"), device="cuda")
    dW = torch.empty(K, N, device="cuda")
    db = torch.empty(N, device="cuda")
    call("rs_dense_bwd_weight", s, ptr(Xb), ldx, ptr(dY), N, ptr(Yc), N, act, M, K, N, ptr(dW),
         ptr(db), 0, ptr(ws), ws_n)
    torch.cuda.synchronize()
    assert_close(to_np(dXb[:, :K]), (dZ @ Wd.T + 0.25).cpu().numpy(), 1e-7 * N * 0.05 * 8, 1e-5,
                 what="dX")
    assert torch.all(dXb[:, K:] == 0.25)
    assert_close(to_np(dW), (Xd.T @ dZ).cpu().numpy(), 1e-7 * M * 0.25 * 8, 1e-5, what="dW")
    assert_close(to_np(db), dZ.sum(0).cpu().numpy(), 1e-7 * M * 8, 1e-5, what="db")


@pytest.mark.parametrize("acc", [False, True])
def test_grouped_dense_matches_layers(acc):
    """grouped_dense (rs_dense_*_grouped: one launch per pass for up to 8 layers) == the layers
    called one by one: mixed shapes and activations, column-slice inputs (row stride > width), a
    weight gradient that splits its reduction, ragged N, gradients accumulated into .grad."""
    from recommendsystem_amd.layers import Dense, grouped_dense
    torch.manual_seed(5)
    M = 2048
    src = torch.randn(M, 256 + 128 + 64, device=DEV)
    specs = [(256, "sigmoid", src[:, :256]), (128, "relu", src[:, 256:384]),
             (3, None, src[:, 384:448]), (64, "relu", torch.randn(M, 32, device=DEV))]
    outs = {}
    for mode in ("single", "grouped"):
        layers = []
        for i, (u, a, x) in enumerate(specs):
            l = Dense(u, a, seed=40 + i, device=DEV)
            l.build(tuple(x.shape), device=DEV)
            with torch.no_grad():
                l.bias.uniform_(-0.2, 0.2, generator=torch.Generator(device=DEV).manual_seed(i))
            if acc:
                l.kernel.grad = torch.full_like(l.kernel, 0.5)
                l.bias.grad = torch.full_like(l.bias, 0.25)
            layers.append(l)
        xs = [x.detach().clone().requires_grad_(True) for _, _, x in specs]
        ys = grouped_dense(layers, xs) if mode == "grouped" else [l(x) for l, x in zip(layers, xs)]
        g = torch.Generator(device=DEV).manual_seed(9)
        loss = sum((y * torch.randn(y.shape, device=DEV, generator=g)).sum() for y in ys)
        loss.backward()
        torch.cuda.synchronize()
        outs[mode] = ([y.detach() for y in ys], [x.grad for x in xs],
                      [l.kernel.grad.clone() for l in layers], [l.bias.grad.clone() for l in layers])
    for what, a, b in zip(("y", "dx", "dW", "db"), outs["grouped"], outs["single"]):
        for i, (u, v) in enumerate(zip(a, b)):
            scale = float(v.abs().max()) + 1e-6
            assert_close(to_np(u), to_np(v), 2e-6 * scale + 1e-6, 1e-5, what=f"{what}[{i}]")


def test_gated_group_matches_gated():
    """gated_group (rs_mul_*_grouped, one launch per pass) == gated per pair: column-slice
    operands, outputs and both gradients bitwise (the same single multiply per element)."""
    from recommendsystem_amd.towers import gated, gated_group
    torch.manual_seed(3)
    src = torch.randn(1000, 256 + 128 + 128, device=DEV)
    gts = torch.rand(1000, 512, device=DEV)
    pairs = [(src[:, :256], gts[:, :256]), (src[:, 256:384], gts[:, 256:384]), (src[:, 384:], gts[:, 384:])]
    res = {}
    for mode in ("single", "group"):
        ds = [d.detach().clone().requires_grad_(True) for d, _ in pairs]
        gs = [g.detach().clone().requires_grad_(True) for _, g in pairs]
        ys = gated_group(ds, gs, 2.0) if mode == "group" else [gated(d, g, 2.0) for d, g in zip(ds, gs)]
        gen = torch.Generator(device=DEV).manual_seed(4)
        sum((y * torch.randn(y.shape, device=DEV, generator=gen)).sum() for y in ys).backward()
        res[mode] = [y.detach() for y in ys] + [d.grad for d in ds] + [g.grad for g in gs]
    for a, b in zip(res["group"], res["single"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,K,N,act", [(2048, 256, 128, 1), (2048, 1712, 960, 1), (300, 64, 48, 2),
                                       (2048, 64, 3, 0)])
def test_dense_bwd_one_launch_equals_two(M, K, N, act):
    """rs_dense_bwd (data + weight gradient blocks in one launch) == rs_dense_bwd_data followed by
    rs_dense_bwd_weight, bitwise (same block plans, same summation order), with accumulation.  A
    shape on the library route (rs_dense_uses_library; the data gradient of rs_dense_bwd then
    reads the materialised dZ, rs_dense_bwd_data's recomputes it on the engine) agrees to fp32
    rounding instead."""
    from recommendsystem_amd import _lib
    from recommendsystem_amd._lib import call, ptr, stream_handle
    lib_route = bool(_lib.load().rs_dense_uses_library(M, K, N))
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    s = stream_handle()
    X = torch.rand(M, K, device="cuda", generator=g) - 0.5
    W = torch.rand(K, N, device="cuda", generator=g) - 0.5
    Y = torch.rand(M, N, device="cuda", generator=g) - 0.3
    dY = torch.rand(M, N, device="cuda", generator=g) - 0.5
    ws_n = int(_lib.load().rs_dense_bwd_weight_workspace_floats(M, K, N))
    res = []
    for one in (True, False):
        ws = torch.full((max(ws_n, 1),), float("nan"), device="cuda")
        dX = torch.full((M, K), 0.5, device="cuda")
        dW = torch.full((K, N), 0.25, device="cuda")
        db = torch.full((N,), 0.125, device="cuda")
        if one:
            call("rs_dense_bwd", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, ptr(W), M, K, N, ptr(dX), K, 1,
                 ptr(dW), ptr(db), 1, ptr(ws), ws_n)
        else:
            call("rs_dense_bwd_data", s, ptr(dY), N, ptr(Y), N, act, ptr(W), M, K, N, ptr(dX), K, 1)
            call("rs_dense_bwd_weight", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, M, K, N, ptr(dW),
                 ptr(db), 1, ptr(ws), ws_n)
        torch.cuda.synchronize()
        res.append((dX, dW, db))
    for a, b in zip(*res):
        if lib_route:
            assert_close(to_np(a), to_np(b), 1e-7 * max(K, N) * 8, 1e-5, what="one vs two (library)")
        else:
            assert torch.equal(a, b)


@pytest.mark.parametrize("M,K,N,act", [(2048, 1712, 960, 1), (4096, 1616, 273, 0), (2048, 1840, 400, 2),
                                       (2048, 1712, 256, 1), (2085, 530, 333, 1), (4096, 1600, 32, 0),
                                       (300, 4096, 600, 1), (2048, 1024, 512, 1), (2048, 1456, 22, 1)])
def test_dense_big_route_matches_engine(M, K, N, act):
    """The large-GEMM kernels (gemm_big.hip; the child forces them down to 2^25 multiply-adds,
    RS_GEMM_BIG_MACS, below their default 2^29 bar) against the engine forced by
    RS_GEMM_BIG=0 and the hipBLASLt route (RS_GEMM_BLAS=1), each in a child process, and all
    against float64: forward (bias + activation), rs_dense_bwd (dX accumulated, dW / db
    accumulated; split-K weight gradients, ragged and unaligned extents: N = 273 / 333 rows take
    the 4-B DMA path, K % 128 == 0 puts db in a tile row of its own), repeated launches bitwise
    equal."""
    import subprocess, sys
    from recommendsystem_amd import _lib
    if M * K * N < (1 << 25):
        pytest.skip("below the large-GEMM kernels' smallest threshold")
    code = f"""
import sys, torch, numpy as np
sys.path.insert(0, {repr(ROOT)})
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle
M, K, N, act = {M}, {K}, {N}, {act}
g = torch.Generator(device="cuda").manual_seed(M + K + N)
X = torch.rand(M, K, device="cuda", generator=g) - 0.5
W = (torch.rand(K, N, device="cuda", generator=g) - 0.5) * 0.1
b = torch.rand(N, device="cuda", generator=g) - 0.5
dY = torch.rand(M, N, device="cuda", generator=g) - 0.5
s = stream_handle()
outs = []
for rep in range(2):
    Y = torch.empty(M, N, device="cuda")
    call("rs_dense_fwd", s, ptr(X), M, K, K, ptr(W), ptr(b), N, act, ptr(Y), N)
    wsn = int(_lib.load().rs_dense_bwd_weight_workspace_floats(M, K, N))
    ws = torch.full((max(wsn, 1),), float("nan"), device="cuda")
    dX = torch.full((M, K), 0.5, device="cuda")
    dW = torch.full((K, N), 0.25, device="cuda")
    db = torch.full((N,), 0.125, device="cuda")
    call("rs_dense_bwd", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, ptr(W), M, K, N, ptr(dX), K, 1,
         ptr(dW), ptr(db), 1, ptr(ws), wsn)
    torch.cuda.synchronize()
    outs.append([t.cpu() for t in (Y, dX, dW, db)])
assert all(torch.equal(a, b) for a, b in zip(*outs))
np.savez(sys.argv[1], *[t.numpy() for t in outs[0]])
"""
    import tempfile
    res = {}
    for mode in ("big", "engine", "lib"):
        env = dict(os.environ)
        env.pop("RS_GEMM_BIG", None)
        env.pop("RS_GEMM_BLAS", None)
        env.pop("RS_GEMM_BIG_MACS", None)
        if mode == "big":  # every product of the shape on the large-GEMM kernels
            env["RS_GEMM_BIG_MACS"] = str(1 << 25)
        if mode == "engine":
            env["RS_GEMM_BIG"] = "0"
        if mode == "lib":
            env["RS_GEMM_BLAS"] = "1"
        with tempfile.NamedTemporaryFile(suffix=".npz") as f:
            r = subprocess.run([sys.executable, "-c", code, f.name], env=env, capture_output=True,
                               text=True, timeout=120)
            assert r.returncode == 0, r.stderr[-3000:]
            z = np.load(f.name)
            res[mode] = [z[f"arr_{i}"] for i in range(4)]
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    X = (torch.rand(M, K, device="cuda", generator=g) - 0.5).double()
    W = ((torch.rand(K, N, device="cuda", generator=g) - 0.5) * 0.1).double()
    b = (torch.rand(N, device="cuda", generator=g) - 0.5).double()
    dY = (torch.rand(M, N, device="cuda", generator=g) - 0.5).double()
    z = X @ W + b
    Y = torch.relu(z) if act == 1 else torch.sigmoid(z) if act == 2 else z
    Yf = torch.from_numpy(res["big"][0]).cuda().double()
    dZ = dY * (Yf > 0) if act == 1 else dY * Yf * (1 - Yf) if act == 2 else dY
    ref = [Y, dZ @ W.T + 0.5, X.T @ dZ + 0.25, dZ.sum(0) + 0.125]
    tols = [1e-7 * K * 0.25 * 8, 1e-7 * N * 0.05 * 8, 1e-7 * M * 0.25 * 8, 1e-7 * M * 8]
    for i, what in enumerate(("y", "dX", "dW", "db")):
        for mode in ("big", "engine", "lib"):
            assert_close(res[mode][i], ref[i].cpu().numpy(), tols[i], 1e-5, what=f"{what} ({mode})")
