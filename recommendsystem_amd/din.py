"""Behaviour-sequence attention pooling layers on librecsys_amd.so.

    DIN          din.py:6-47               DIN(**kwargs)(queries [B,H], keys [B,T,H],
                                           values [B,T,H], seq_length [B]) -> [B,H]
                                           ReLU-MLP scores masked to 0, no softmax.
    StaytimeDIN  staytime/layer.py:6-41    DIN(**kwargs)(query [B,H], facts [B,T,H],
                                           mask [B,>=T] bool) -> [B,H]
                                           masked (-2**32+1) softmax over T.

Both build their two Dense layers on the first call (din_nn_0 = Dense(16, relu), din_nn_1 =
Dense(1, relu) | layer_1 = Dense(16, sigmoid), layer_2 = Dense(1)), glorot_uniform kernels and
zero biases, stored as one flat block [W1 | b1 | W2 | b2] so the backward kernel accumulates the
whole weight gradient in place.  Embedding width H = 16 is the compiled shape (configs 4 and 5).
Inputs may be strided views whose last dimension is contiguous (e.g. the [:, :, 0:16] slice of a
32-wide sequence lookup, staytime/VideoDnn.py:68) -- the kernel reads them in place.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle
from .params import FlatBlock, glorot_uniform_, grads_contiguous

VAR_RELU_SUM, VAR_SOFTMAX = 0, 1
HIDDEN = 16


def _rows_view(t: torch.Tensor) -> torch.Tensor:
    """A view the kernel can read in place: fp32, unit stride in the last dim, 16-byte aligned
    row strides; otherwise a contiguous copy."""
    if t.dtype != torch.float32:
        t = t.float()
    ok = t.stride(-1) == 1 and all(s % 4 == 0 for s in t.stride()[:-1]) and t.data_ptr() % 16 == 0
    return t if ok else t.contiguous()


class _DINFn(torch.autograd.Function):
    """cat_q: return [pooled, q] [B, 2H] (the pooled rows written by the kernel into the left
    half); the backward reads d pooled in place and adds the right half's gradient onto the
    query's (rs_din_bwd_ex dq_base) -- no concat gradient slice copy, no separate sum launch."""

    @staticmethod
    def forward(ctx, q, keys, values, lengths, mask, W1, b1, W2, b2, variant, wide=False,
                cat_q=False):
        _lib.require_device(q, keys, values, W1)
        q = _rows_view(q)
        keys = _rows_view(keys)
        # wide: keys [B, T, W > H] whose first H columns are the facts; the backward returns the
        # [B, T, W] gradient (zeros past H) straight from the kernel (rs_din_bwd_strided)
        ctx.wide_w = keys.shape[2] if wide else 0
        if wide:
            keys = keys[:, :, :q.shape[1]]
        same = values is None or values.data_ptr() == keys.data_ptr() and values.shape == keys.shape
        values = keys if same else _rows_view(values)
        B, T, H = keys.shape
        if cat_q:
            buf = torch.empty(B, 2 * H, device=q.device, dtype=torch.float32)
            buf[:, H:].copy_(q)
            out, out_ld = buf[:, :H], 2 * H
        else:
            buf = out = torch.empty(B, H, device=q.device, dtype=torch.float32)
            out_ld = H
        probs = torch.empty(B, T, device=q.device, dtype=torch.float32) if variant == 1 else None
        m8 = mask.view(torch.uint8) if mask is not None else None
        call("rs_din_fwd", stream_handle(), variant, ptr(q), q.stride(0), ptr(keys), keys.stride(0),
             keys.stride(1), ptr(values), values.stride(0), values.stride(1), B, T, H, ptr(lengths),
             ptr(m8), m8.stride(0) if m8 is not None else 0, ptr(W1), ptr(b1), ptr(W2), ptr(b2),
             ptr(out), out_ld, ptr(probs))
        ctx.save_for_backward(q, keys, values, lengths, m8, W1, b1, W2, b2, probs)
        ctx.variant, ctx.same, ctx.cat_q = variant, same, cat_q
        return buf

    @staticmethod
    def backward(ctx, dout):
        q, keys, values, lengths, m8, W1, b1, W2, b2, probs = ctx.saved_tensors
        variant = ctx.variant
        dout = _rows_view(dout)
        B, T, H = keys.shape
        base = dout[:, H:] if ctx.cat_q else None
        dev = q.device
        dq = torch.empty(B, H, device=dev, dtype=torch.float32)
        Wd = ctx.wide_w or H
        dk = torch.empty(B, T, Wd, device=dev, dtype=torch.float32)
        dv = dk if (ctx.same or variant == 1) else torch.empty(B, T, H, device=dev, dtype=torch.float32)
        ws_n = int(_lib.load().rs_din_bwd_workspace_floats(variant, B, T, H))
        ws = torch.empty(max(ws_n, 1), device=dev, dtype=torch.float32)
        params = (W1, b1, W2, b2)
        block = grads_contiguous(params)
        in_place = block is not None
        dparams = block if in_place else torch.empty(sum(p.numel() for p in params), device=dev)
        if ctx.wide_w and not (ctx.same or variant == 1):
            raise NotImplementedError("wide facts need keys == values")
        call("rs_din_bwd_ex", stream_handle(), variant, ptr(q), q.stride(0), ptr(keys),
             keys.stride(0), keys.stride(1), ptr(values), values.stride(0), values.stride(1), B, T,
             H, ptr(lengths), ptr(m8), m8.stride(0) if m8 is not None else 0, ptr(W1), ptr(b1),
             ptr(W2), ptr(b2), ptr(probs), ptr(dout), dout.stride(0), ptr(dq), H,
             ptr(base) if base is not None else None, dout.stride(0), ptr(dk), ptr(dv), Wd, Wd,
             ptr(dparams), 1 if in_place else 0, ptr(ws), ws_n)
        if in_place:
            wgrads = (None, None, None, None)
        else:
            outs, off = [], 0
            for p in params:
                outs.append(dparams[off:off + p.numel()].view(p.shape))
                off += p.numel()
            wgrads = tuple(outs)
        if ctx.same or variant == 1:
            return (dq, dk, None, None, None, *wgrads, None, None, None)
        return (dq, dk, dv, None, None, *wgrads, None, None, None)


class _DINBase(nn.Module):
    VARIANT = VAR_RELU_SUM
    BLOCKS = 3
    ACTS = ("relu", "relu")

    def __init__(self, seed=0, device=None, **kwargs):
        super().__init__()
        self.seed = int(seed)
        self._device = device
        self.built = False
        self.name = kwargs.get("name", "din")

    def build(self, input_shape, device=None):
        H = int(input_shape[-1])
        if _lib.load().rs_din_param_count(self.VARIANT, H) < 0:
            raise NotImplementedError(f"DIN pooling is compiled for embedding width 16, got {H}")
        device = device or self._device or torch.device("cuda")
        K = self.BLOCKS * H
        blk = FlatBlock([(K, HIDDEN), (HIDDEN,), (HIDDEN, 1), (1,)], device)
        self.W1, self.b1, self.W2, self.b2 = blk.params()
        gen = torch.Generator().manual_seed(self.seed)
        glorot_uniform_(self.W1, K, HIDDEN, gen)
        glorot_uniform_(self.W2, HIDDEN, 1, gen)
        self.input_dim = H
        self.built = True

    def _pool(self, q, keys, values, lengths, mask):
        if q.dim() != 2 or keys.dim() != 3 or keys.shape[0] != q.shape[0] or keys.shape[2] != q.shape[1]:
            raise ValueError(f"expected query [B, H] and keys [B, T, H], got {tuple(q.shape)} and "
                             f"{tuple(keys.shape)}")
        if not self.built:
            self.build(tuple(keys.shape), device=keys.device)
        from . import ops
        if ops.custom_ops_enabled():  # torch.ops.ctr.din_pool (traceable, functional grads)
            v = keys if values is None else values
            return torch.ops.ctr.din_pool(q, keys, v, lengths, mask, self.W1, self.b1, self.W2,
                                          self.b2, self.VARIANT)[0]
        return _DINFn.apply(q, keys, values, lengths, mask, self.W1, self.b1, self.W2, self.b2,
                            self.VARIANT)

    def pool_concat(self, q, keys, values=None, lengths=None, mask=None):
        """torch.cat([pool(q, keys, values, lengths, mask), q], dim=1) with the pooled rows
        written into the concat by the kernel and the query's two gradients summed inside the
        backward launch."""
        from . import ops
        if ops.custom_ops_enabled() or q.dim() != 2 or keys.dim() != 3:
            return torch.cat([self._pool(q, keys, values, lengths, mask), q], dim=1)
        if not self.built:
            self.build(tuple(keys.shape), device=keys.device)
        if keys.shape[0] != q.shape[0] or keys.shape[2] != q.shape[1]:
            raise ValueError(f"expected query [B, H] and keys [B, T, H], got {tuple(q.shape)} and "
                             f"{tuple(keys.shape)}")
        return _DINFn.apply(q, keys, values, lengths, mask, self.W1, self.b1, self.W2, self.b2,
                            self.VARIANT, False, True)


class DIN(_DINBase):
    """din.py:6-47.  ``seq_length`` [B] int: positions t >= seq_length[b] get score 0
    (tf.sequence_mask(seq_length), whose maxlen = max(seq_length) must equal T, :24,40-42)."""
    VARIANT, BLOCKS = VAR_RELU_SUM, 3

    def forward(self, queries, keys, values, seq_length=None):
        lengths = None
        if seq_length is not None:
            lengths = seq_length.reshape(-1).to(device=keys.device, dtype=torch.int32).contiguous()
        if values.shape != keys.shape:
            raise ValueError("keys and values must have the same shape [B, T, H]")
        return self._pool(queries, keys, values, lengths, None)

    def forward_concat(self, queries, keys, values, seq_length=None):
        """torch.cat([self(queries, keys, values, seq_length), queries], dim=1) (the config-4
        head input, din.py's pooled output next to its query) via pool_concat."""
        lengths = None
        if seq_length is not None:
            lengths = seq_length.reshape(-1).to(device=keys.device, dtype=torch.int32).contiguous()
        if values.shape != keys.shape:
            raise ValueError("keys and values must have the same shape [B, T, H]")
        return self.pool_concat(queries, keys, values, lengths, None)


class StaytimeDIN(_DINBase):
    """staytime/layer.py:6-41 (imported there as ``DIN``).  ``mask`` [B, >=T] bool is sliced to
    the first T columns (:30); masked positions take the score -2**32+1 before the softmax, so a
    fully masked row pools the facts uniformly."""
    VARIANT, BLOCKS = VAR_SOFTMAX, 4

    def forward(self, query, facts, mask=None, wide=False):
        """``wide``: facts [B, T, W] (W <= 2 * H) whose first H = query width columns are the
        sequence embedding (the staytime 32-wide sequence rows, VideoDnn.py:57-77); no slice."""
        m = None
        if mask is not None:
            if mask.dim() != 2 or mask.shape[0] != facts.shape[0] or mask.shape[1] < facts.shape[1]:
                raise ValueError("mask must be [B, >= T]")
            m = mask.to(device=facts.device, dtype=torch.bool)
            if m.stride(-1) != 1:
                m = m.contiguous()
        if wide:
            if not self.built:
                self.build((1, facts.shape[1], query.shape[1]), device=facts.device)
            return _DINFn.apply(query, facts, None, None, m, self.W1, self.b1, self.W2, self.b2,
                                self.VARIANT, True)
        return self._pool(query, facts, None, None, m)
