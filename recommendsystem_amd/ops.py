"""PyTorch custom operators (torch.library) over the C ABI: ``torch.ops.ctr.*`` (SURVEY §8(b),
north_star "hosted from Python via PyTorch-ROCm custom ops").

Each op is functional (new outputs, no aliasing), has a fake (meta) implementation for
FakeTensor / torch.compile tracing, and the differentiable ones register their autograd formula
through a companion backward op, so graphs captured by dynamo / AOTAutograd keep calling the HIP
kernels:

    ctr::interacting_fwd / ctr::interacting_bwd   InteractingLayer.call (InteractingLayer.py:37-61)
    ctr::din_pool / ctr::din_pool_bwd             DIN.call (din.py:18-47) and staytime DIN.call
                                                  (staytime/layer.py:16-41)
    ctr::dense / ctr::dense_bwd                   tf.keras.layers.Dense(units, activation)
    ctr::embedding_lookup                         EmbeddingFeatures forward (rank/ctr/base_model.py:
                                                  203-217); its sparse push is the table's
                                                  (embedding.SparseTable), not an autograd output

The layer classes (layers.InteractingLayer, din.DIN, layers.Dense) keep their in-place gradient
fast path (autograd.Function writing into the flat parameter block); ``use_custom_ops(True)``
routes them through these ops instead (functional gradients; traceable).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib
from ._lib import call, ptr, stream_handle

_U64 = 0xFFFFFFFFFFFFFFFF
_USE = {"on": False}


def use_custom_ops(on: bool = True) -> None:
    """Route InteractingLayer / DIN / Dense forward through torch.ops.ctr (traceable)."""
    _USE["on"] = bool(on)


def custom_ops_enabled() -> bool:
    return _USE["on"]


def _seed(s: int) -> int:
    return int(s) & _U64


def _signed(s: int) -> int:
    """uint64 seed -> the int64 a torch schema `int` carries."""
    s = int(s) & _U64
    return s - (1 << 64) if s >= (1 << 63) else s


# ============================================================================================
# InteractingLayer
# ============================================================================================
@custom_op("ctr::interacting_fwd", mutates_args=())
def interacting_fwd(x: Tensor, W: Tensor, bias: Tensor, gamma: Tensor, beta: Tensor,
                    layer_num: int, head_num: int, use_res: bool, eps: float, drop_rate: float,
                    seed: int) -> tuple[Tensor, Tensor, Tensor]:
    """Returns (y, xsave, asave): asave is the saved pair's attention save (rs_il_fwd_saved;
    empty for shapes without one), consumed by interacting_bwd."""
    _lib.require_device(x, W)
    x = x.contiguous().float()
    B, F, E = x.shape
    U = W.shape[1] // 4
    y = torch.empty(B, F, U, device=x.device)
    xsave = torch.empty(max(layer_num - 1, 0), B, F, U, device=x.device)
    n_save = int(_lib.load().rs_il_attn_save_floats(B, F, U, head_num, layer_num))
    asave = torch.empty(n_save, device=x.device)
    call("rs_il_fwd_saved", stream_handle(), ptr(x), B, F, E, U, head_num, layer_num, ptr(W),
         ptr(bias), ptr(gamma), ptr(beta), eps, int(use_res), drop_rate, _seed(seed), ptr(y), F * U,
         ptr(xsave) if layer_num > 1 else None, ptr(asave) if n_save else None, n_save)
    return y, xsave, asave


@interacting_fwd.register_fake
def _(x, W, bias, gamma, beta, layer_num, head_num, use_res, eps, drop_rate, seed):
    B, F, _ = x.shape
    U = W.shape[1] // 4
    n_save = int(_lib.load().rs_il_attn_save_floats(B, F, U, head_num, layer_num))
    return (x.new_empty(B, F, U), x.new_empty(max(layer_num - 1, 0), B, F, U),
            x.new_empty(n_save))


@custom_op("ctr::interacting_bwd", mutates_args=())
def interacting_bwd(dy: Tensor, x: Tensor, xsave: Tensor, asave: Tensor, W: Tensor, bias: Tensor,
                    gamma: Tensor, beta: Tensor, layer_num: int, head_num: int, use_res: bool,
                    eps: float, drop_rate: float,
                    seed: int) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    x = x.contiguous().float()
    dy = dy.contiguous().float()
    B, F, E = x.shape
    U = W.shape[1] // 4
    dx = torch.empty_like(x)
    ws_n = int(_lib.load().rs_il_bwd_workspace_floats(B, E, U))
    ws = torch.empty(max(ws_n, 1), device=x.device)
    n = W.numel() + bias.numel() + gamma.numel() + beta.numel()
    dp = torch.empty(n, device=x.device)
    call("rs_il_bwd_saved", stream_handle(), ptr(x), ptr(xsave) if layer_num > 1 else None, ptr(dy),
         F * U, B, F, E, U, head_num, layer_num, ptr(W), ptr(bias), ptr(gamma), ptr(beta), eps,
         int(use_res), drop_rate, _seed(seed), ptr(dx), 0, ptr(dp), 0, ptr(ws), ws_n,
         ptr(asave) if asave.numel() else None, asave.numel())
    o1, o2, o3 = W.numel(), W.numel() + bias.numel(), W.numel() + bias.numel() + gamma.numel()
    return (dx, dp[:o1].view(W.shape).clone(), dp[o1:o2].clone(), dp[o2:o3].clone(),
            dp[o3:].clone())


@interacting_bwd.register_fake
def _(dy, x, xsave, asave, W, bias, gamma, beta, layer_num, head_num, use_res, eps, drop_rate, seed):
    return (torch.empty_like(x), torch.empty_like(W), torch.empty_like(bias),
            torch.empty_like(gamma), torch.empty_like(beta))


def _il_setup(ctx, inputs, output):
    x, W, bias, gamma, beta, L, H, res, eps, rate, seed = inputs
    ctx.save_for_backward(x, output[1], output[2], W, bias, gamma, beta)
    ctx.cfg = (L, H, res, eps, rate, seed)


def _il_backward(ctx, dy, _dxsave, _dasave):
    x, xsave, asave, W, bias, gamma, beta = ctx.saved_tensors
    L, H, res, eps, rate, seed = ctx.cfg
    dx, dW, db, dg, dbe = torch.ops.ctr.interacting_bwd(dy, x, xsave, asave, W, bias, gamma, beta,
                                                        L, H, res, eps, rate, seed)
    return dx, dW, db, dg, dbe, None, None, None, None, None, None


interacting_fwd.register_autograd(_il_backward, setup_context=_il_setup)


def interacting_layer(x, W, bias, gamma, beta, layer_num=1, head_num=1, use_res=True, eps=1e-14,
                      drop_rate=0.0, seed=0):
    """Functional InteractingLayer (torch.ops.ctr.interacting_fwd); returns [B, F, U]."""
    return torch.ops.ctr.interacting_fwd(x, W, bias, gamma, beta, int(layer_num), int(head_num),
                                         bool(use_res), float(eps), float(drop_rate),
                                         _signed(seed))[0]


# ============================================================================================
# DIN pools
# ============================================================================================
@custom_op("ctr::din_pool", mutates_args=())
def din_pool(q: Tensor, keys: Tensor, values: Tensor, lengths: Optional[Tensor],
             mask: Optional[Tensor], W1: Tensor, b1: Tensor, W2: Tensor, b2: Tensor,
             variant: int) -> tuple[Tensor, Tensor]:
    """variant 0: din.py relu-sum (lengths int32 [B] or None); 1: staytime masked softmax
    (mask bool [B, >=T] or None) over the facts = keys (values is not read: staytime's DIN
    pools the facts it scores, staytime/layer.py:36-41; its gradient is zero).
    Returns (out [B, H], probs [B, T] (variant 1) / [0])."""
    _lib.require_device(q, keys, W1)
    q, keys = q.contiguous().float(), keys.contiguous().float()
    values = keys if variant == 1 else values.contiguous().float()
    B, T, H = keys.shape
    out = torch.empty(B, H, device=q.device)
    probs = torch.empty(B, T, device=q.device) if variant == 1 else torch.empty(0, device=q.device)
    m8 = mask.contiguous().view(torch.uint8) if mask is not None else None
    lens = lengths.to(torch.int32).contiguous() if lengths is not None else None
    call("rs_din_fwd", stream_handle(), variant, ptr(q), H, ptr(keys), T * H, H, ptr(values), T * H, H,
         B, T, H, ptr(lens), ptr(m8), m8.stride(0) if m8 is not None else 0, ptr(W1), ptr(b1),
         ptr(W2), ptr(b2), ptr(out), H, ptr(probs) if variant == 1 else None)
    return out, probs


@din_pool.register_fake
def _(q, keys, values, lengths, mask, W1, b1, W2, b2, variant):
    B, T, H = keys.shape
    return q.new_empty(B, H), q.new_empty(B, T) if variant == 1 else q.new_empty(0)


@custom_op("ctr::din_pool_bwd", mutates_args=())
def din_pool_bwd(dout: Tensor, q: Tensor, keys: Tensor, values: Tensor, lengths: Optional[Tensor],
                 mask: Optional[Tensor], W1: Tensor, b1: Tensor, W2: Tensor, b2: Tensor,
                 probs: Tensor, variant: int) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor,
                                                        Tensor, Tensor]:
    q, keys = q.contiguous().float(), keys.contiguous().float()
    values = keys if variant == 1 else values.contiguous().float()
    dout = dout.contiguous().float()
    B, T, H = keys.shape
    dev = q.device
    dq = torch.empty(B, H, device=dev)
    dk = torch.empty(B, T, H, device=dev)
    dv = torch.empty(B, T, H, device=dev) if variant == 0 else dk
    m8 = mask.contiguous().view(torch.uint8) if mask is not None else None
    lens = lengths.to(torch.int32).contiguous() if lengths is not None else None
    ws_n = int(_lib.load().rs_din_bwd_workspace_floats(variant, B, T, H))
    ws = torch.empty(max(ws_n, 1), device=dev)
    n = W1.numel() + b1.numel() + W2.numel() + b2.numel()
    dp = torch.empty(n, device=dev)
    call("rs_din_bwd", stream_handle(), variant, ptr(q), H, ptr(keys), T * H, H, ptr(values), T * H,
         H, B, T, H, ptr(lens), ptr(m8), m8.stride(0) if m8 is not None else 0, ptr(W1), ptr(b1),
         ptr(W2), ptr(b2), ptr(probs) if variant == 1 else None, ptr(dout), H, ptr(dq), H, ptr(dk),
         ptr(dv), ptr(dp), 0, ptr(ws), ws_n)
    if variant == 1:  # staytime: values are the facts (= keys), dk holds the whole gradient
        dv = torch.zeros_like(dk)
    o = [W1.numel(), b1.numel(), W2.numel(), b2.numel()]
    s = [0, o[0], o[0] + o[1], o[0] + o[1] + o[2], n]
    return (dq, dk, dv, dp[s[0]:s[1]].view(W1.shape).clone(), dp[s[1]:s[2]].clone(),
            dp[s[2]:s[3]].view(W2.shape).clone(), dp[s[3]:s[4]].clone())


@din_pool_bwd.register_fake
def _(dout, q, keys, values, lengths, mask, W1, b1, W2, b2, probs, variant):
    return (torch.empty_like(q), torch.empty_like(keys), torch.empty_like(values),
            torch.empty_like(W1), torch.empty_like(b1), torch.empty_like(W2), torch.empty_like(b2))


def _din_setup(ctx, inputs, output):
    q, keys, values, lengths, mask, W1, b1, W2, b2, variant = inputs
    ctx.save_for_backward(q, keys, values, lengths, mask, W1, b1, W2, b2, output[1])
    ctx.variant = variant


def _din_backward(ctx, dout, _dprobs):
    q, keys, values, lengths, mask, W1, b1, W2, b2, probs = ctx.saved_tensors
    dq, dk, dv, dW1, db1, dW2, db2 = torch.ops.ctr.din_pool_bwd(
        dout, q, keys, values, lengths, mask, W1, b1, W2, b2, probs, ctx.variant)
    return dq, dk, dv, None, None, dW1, db1, dW2, db2, None


din_pool.register_autograd(_din_backward, setup_context=_din_setup)


# ============================================================================================
# Dense
# ============================================================================================
@custom_op("ctr::dense", mutates_args=())
def dense(x: Tensor, W: Tensor, b: Tensor, act: int) -> Tensor:
    """tf.keras.layers.Dense on [M, K] rows: act 0 linear, 1 relu, 2 sigmoid."""
    _lib.require_device(x, W)
    x = x.contiguous().float()
    M, K = x.shape
    N = W.shape[1]
    y = torch.empty(M, N, device=x.device)
    call("rs_dense_fwd", stream_handle(), ptr(x), M, K, K, ptr(W), ptr(b), N, act, ptr(y), N)
    return y


@dense.register_fake
def _(x, W, b, act):
    return x.new_empty(x.shape[0], W.shape[1])


@custom_op("ctr::dense_bwd", mutates_args=())
def dense_bwd(dy: Tensor, x: Tensor, y: Tensor, W: Tensor, act: int) -> tuple[Tensor, Tensor, Tensor]:
    x, y, dy = x.contiguous().float(), y.contiguous().float(), dy.contiguous().float()
    M, K = x.shape
    N = W.shape[1]
    s = stream_handle()
    dx = torch.empty_like(x)
    call("rs_dense_bwd_data", s, ptr(dy), N, ptr(y), N, act, ptr(W), M, K, N, ptr(dx), K, 0)
    ws_n = int(_lib.load().rs_dense_bwd_weight_workspace_floats(M, K, N))
    ws = torch.empty(max(ws_n, 1), device=x.device)
    dW = torch.empty_like(W)
    db = torch.empty(N, device=x.device)
    call("rs_dense_bwd_weight", s, ptr(x), K, ptr(dy), N, ptr(y), N, act, M, K, N, ptr(dW), ptr(db),
         0, ptr(ws), ws_n)
    return dx, dW, db


@dense_bwd.register_fake
def _(dy, x, y, W, act):
    return torch.empty_like(x), torch.empty_like(W), W.new_empty(W.shape[1])


def _dense_setup(ctx, inputs, output):
    x, W, b, act = inputs
    ctx.save_for_backward(x, output, W)
    ctx.act = act


def _dense_backward(ctx, dy):
    x, y, W = ctx.saved_tensors
    dx, dW, db = torch.ops.ctr.dense_bwd(dy, x, y, W, ctx.act)
    return dx, dW, db, None


dense.register_autograd(_dense_backward, setup_context=_dense_setup)


# ============================================================================================
# embedding lookup (forward only; the push belongs to SparseTable)
# ============================================================================================
@custom_op("ctr::embedding_lookup", mutates_args=())
def embedding_lookup(ids: Tensor, offsets: Optional[Tensor], row_base: Tensor, bucket: Tensor,
                     hash_mode: int, combiner: int, table: Tensor) -> tuple[Tensor, Tensor]:
    """(out [B, F, dim], rows int32 [nnz]) for ids [B, F] (offsets None) or ids [nnz] +
    offsets int32 [B*F + 1]."""
    _lib.require_device(ids, table)
    F = row_base.numel()
    ids = ids.contiguous()
    B = ids.shape[0] if offsets is None else (offsets.numel() - 1) // F
    dim = table.shape[1]
    out = torch.empty(B, F, dim, device=table.device)
    rows = torch.empty(ids.numel(), device=table.device, dtype=torch.int32)
    offs = offsets.to(torch.int32).contiguous() if offsets is not None else None
    call("rs_embedding_lookup_fwd", stream_handle(), ptr(ids), ptr(offs), B, F, ptr(row_base),
         ptr(bucket), hash_mode, combiner, ptr(table), table.shape[0], dim, ptr(out), F * dim, dim,
         ptr(rows))
    return out, rows


@embedding_lookup.register_fake
def _(ids, offsets, row_base, bucket, hash_mode, combiner, table):
    F = row_base.shape[0]
    if offsets is None:
        B = ids.shape[0]
    else:
        B = (offsets.shape[0] - 1) // F
    return table.new_empty(B, F, table.shape[1]), ids.new_empty(ids.numel(), dtype=torch.int32)
