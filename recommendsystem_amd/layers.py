"""Drop-in layers for the CTR feature-interaction path, keeping the reference's constructor
kwargs, call signatures and error messages; every compute step runs in librecsys_amd.so.

    InteractingLayer   InteractingLayer.py:7-61 (== rank/multi_head/interacting_layer.py)
    Dense              tf.keras.layers.Dense(units, activation) as used on the path
    MultiLayerDense    common_module.multi_dense_layer.MultiLayerDense (absent from the reference;
                       pinned: sequential Dense(u, activation) for every u, SURVEY §8c decision 2)

Layers are torch.nn.Modules.  Like Keras, parameters are created on the first call from the
input's last dimension (or by an explicit ``build(input_shape)``).  Gradients: when a layer's
``.grad`` tensors live in one flat block (always, unless the caller replaced them), the backward
kernels accumulate into them in place and autograd receives ``None`` for the weights -- no extra
accumulate kernels.  Otherwise the gradients are returned to autograd normally.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle
from .params import FlatBlock, glorot_uniform_, grads_contiguous

ACTIVATIONS = {None: 0, "linear": 0, "relu": 1, "sigmoid": 2}


def _act_code(activation) -> int:
    if activation in ACTIVATIONS:
        return ACTIVATIONS[activation]
    raise NotImplementedError(f"activation {activation!r} is not on the fused path "
                              f"(supported: {sorted(k for k in ACTIVATIONS if k)})")


# ============================================================================================
# InteractingLayer
# ============================================================================================
class GradSink:
    """Hands one consumer's input gradient to another consumer of the same input so the second
    one's backward ADDS its share in its own launch (rs_dense_bwd with dx accumulate) instead of
    autograd summing two [B, K] gradients with an extra elementwise launch.  The producer's
    backward must run first: it does whenever the producer sits downstream of the consumer in
    the forward (the interacting layer's concat takes the deep tower's output)."""

    __slots__ = ("buf",)

    def __init__(self):
        self.buf = None


class _InteractingFn(torch.autograd.Function):
    """lead: None -> y [B, F, U]; a [B, Dl] tensor -> the concat [lead | y.reshape(B, F U)]
    [B, Dl + F U] with y written in place by the kernel (y_ld) and its backward reading its dy
    slice in place (dy_ld): no concat copy forward, no contiguous copy of the split gradient."""

    @staticmethod
    def forward(ctx, x, W, bias, gamma, beta, layer, seed, drop_rate, lead=None, sink=None):
        _lib.require_device(x, W)
        x = x.contiguous()
        B, F, E = x.shape
        U, H, L = layer.unit_num, layer.head_num, layer.layer_num
        if lead is not None:
            Dl = lead.shape[1]
            out = torch.empty(B, Dl + F * U, device=x.device, dtype=torch.float32)
            out[:, :Dl].copy_(lead)
            y, y_ld = out[:, Dl:], Dl + F * U
        else:
            Dl = 0
            y = out = torch.empty(B, F, U, device=x.device, dtype=torch.float32)
            y_ld = F * U
        xsave = torch.empty(max(L - 1, 0), B, F, U, device=x.device, dtype=torch.float32)
        # many-field shapes (F > 64): the forward also saves the attention output, softmax stats
        # and dropout bits so the backward does not recompute them (rs_il_fwd_saved)
        n_save = int(_lib.load().rs_il_attn_save_floats(B, F, U, H, L))
        asave = torch.empty(n_save, device=x.device, dtype=torch.float32)
        call("rs_il_fwd_saved", stream_handle(), ptr(x), B, F, E, U, H, L, ptr(W), ptr(bias),
             ptr(gamma), ptr(beta), layer.epsilon, int(layer.use_res), drop_rate, seed, ptr(y),
             y_ld, ptr(xsave) if L > 1 else None, ptr(asave) if n_save else None, n_save)
        ctx.save_for_backward(x, xsave, W, bias, gamma, beta, asave)
        ctx.layer, ctx.seed, ctx.drop_rate, ctx.Dl = layer, seed, drop_rate, Dl
        ctx.has_lead = lead is not None
        ctx.sink = sink
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xsave, W, bias, gamma, beta, asave = ctx.saved_tensors
        layer = ctx.layer
        B, F, E = x.shape
        U, H, L = layer.unit_num, layer.head_num, layer.layer_num
        Dl = ctx.Dl
        if ctx.has_lead:
            if dout.stride(1) != 1 or dout.stride(0) % 4 or dout.dtype != torch.float32:
                dout = dout.contiguous().float()
            d_lead = dout[:, :Dl]
            dy, dy_ld = dout[:, Dl:], dout.stride(0)
        else:
            d_lead = None
            dy, dy_ld = dout.contiguous(), F * U
        dx = torch.empty_like(x)
        ws_n = int(_lib.load().rs_il_bwd_workspace_floats(B, E, U))
        ws = torch.empty(ws_n, device=x.device, dtype=torch.float32)
        params = (W, bias, gamma, beta)
        block = grads_contiguous(params)
        in_place = block is not None
        dparams = block if in_place else torch.empty(
            sum(p.numel() for p in params), device=x.device, dtype=torch.float32)
        call("rs_il_bwd_saved", stream_handle(), ptr(x), ptr(xsave) if L > 1 else None, ptr(dy),
             dy_ld, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), layer.epsilon,
             int(layer.use_res), ctx.drop_rate, ctx.seed, ptr(dx), 0, ptr(dparams),
             1 if in_place else 0, ptr(ws), ws_n, ptr(asave) if asave.numel() else None,
             asave.numel())
        if ctx.sink is not None:  # the deep tower's first Dense adds its dx onto this one
            ctx.sink.buf, dx = dx.view(B, F * E), None
        if in_place:
            return dx, None, None, None, None, None, None, None, d_lead, None
        outs, off = [], 0
        for p in params:
            outs.append(dparams[off:off + p.numel()].view(p.shape))
            off += p.numel()
        return (dx, *outs, None, None, None, d_lead, None)


class InteractingLayer(nn.Module):
    """AutoInt interacting layer, InteractingLayer.py:7-61.

    Same kwargs/defaults as the reference (:9-16).  ``ln_epsilon`` pins the epsilon of the
    missing ``layer_normalization.LayerNormalization`` (keras-layer-normalization default
    K.epsilon()**2 = 1e-14; SURVEY §8c open decision 1).  ``seed`` seeds the counter-based
    dropout mask (InteractingLayer.py:53-54; active only in training mode with use_dropout).
    """

    def __init__(self, layer_num=1, unit_num=128, head_num=1, use_dropout=False, dropout_rate=0.3,
                 use_res=True, ln_epsilon=1e-14, seed=0, device=None, **kwargs):
        super().__init__()
        self.layer_num = int(layer_num)
        self.unit_num = int(unit_num)
        self.head_num = int(head_num)
        self.use_dropout = bool(use_dropout)
        self.dropout_rate = float(dropout_rate)
        self.use_res = bool(use_res)
        self.epsilon = float(ln_epsilon)
        self.seed = int(seed)
        self._calls = 0
        self._device = device
        self.built = False
        self.name = kwargs.get("name", "interacting_layer")

    # Keras Layer.build (InteractingLayer.py:33-35) + the Dense builds it triggers
    def build(self, input_shape, device=None):
        if len(input_shape) != 3:
            raise ValueError('The rank of input of InteractingLayer must be 3, but now is %d'
                             % len(input_shape))
        E, U, H = int(input_shape[-1]), self.unit_num, self.head_num
        if U % H != 0:  # tf.split(query, head_num, axis=2) (InteractingLayer.py:47)
            raise ValueError(f"Dimension size must be evenly divisible by {H} but is {U}")
        if self.layer_num > 1 and E != U:  # the tied Dense kernels are built for the first input
            raise ValueError(f"layer_num > 1 needs unit_num == input dim (tied weights): "
                             f"unit_num={U}, input dim={E}")
        device = device or self._device or torch.device("cuda")
        blk = FlatBlock([(E, 4 * U), (4 * U,), (U,), (U,)], device)
        self.kernel, self.bias, self.gamma, self.beta = blk.params()
        gen = torch.Generator().manual_seed(self.seed)
        with torch.no_grad():
            for j in range(4):  # query / key / value / res Dense kernels, each glorot_uniform
                k = torch.empty(E, U)
                glorot_uniform_(k, E, U, gen)
                self.kernel[:, j * U:(j + 1) * U].copy_(k)
            self.gamma.fill_(1.0)
        self.input_dim = E
        self.built = True

    # Keras-named views of the fused [E, 4U] kernel
    def dense_kernel(self, which: str) -> torch.Tensor:
        j = {"query": 0, "key": 1, "value": 2, "res": 3}[which]
        return self.kernel[:, j * self.unit_num:(j + 1) * self.unit_num]

    def dense_bias(self, which: str) -> torch.Tensor:
        j = {"query": 0, "key": 1, "value": 2, "res": 3}[which]
        return self.bias[j * self.unit_num:(j + 1) * self.unit_num]

    def forward(self, inputs):
        if inputs.dim() != 3:
            raise ValueError('The rank of input of InteractingLayer must be 3, but now is %d'
                             % inputs.dim())
        if not self.built:
            self.build(tuple(inputs.shape), device=inputs.device)
        drop = self.dropout_rate if (self.use_dropout and self.training) else 0.0
        seed = (self.seed * 1000003 + self._calls) & 0xFFFFFFFFFFFFFFFF
        self._calls += 1
        from . import ops
        if ops.custom_ops_enabled():  # torch.ops.ctr.interacting_fwd (traceable, functional grads)
            return ops.interacting_layer(inputs.float(), self.kernel, self.bias, self.gamma,
                                         self.beta, self.layer_num, self.head_num, self.use_res,
                                         self.epsilon, drop, seed)
        return _InteractingFn.apply(inputs.float(), self.kernel, self.bias, self.gamma, self.beta,
                                    self, seed, drop)

    def forward_concat(self, lead, inputs, grad_sink=None):
        """tf.concat([lead, Flatten()(self(inputs))], axis=1) (rank/multi_head/multidnn.py:71)
        with the layer's output written straight into the concat and its gradient read from
        there in place.  grad_sink: a GradSink shared with the Dense that consumes
        inputs.reshape(B, -1) upstream of `lead` (Dense.forward(x, grad_sink=...)); the layer's
        input gradient then reaches `inputs` through that Dense's backward."""
        if not self.built:
            self.build(tuple(inputs.shape), device=inputs.device)
        from . import ops
        if ops.custom_ops_enabled() or lead.dim() != 2 or lead.shape[1] % 4:
            return torch.cat([lead, self(inputs).reshape(inputs.shape[0], -1)], dim=1)
        if inputs.dim() != 3:
            raise ValueError('The rank of input of InteractingLayer must be 3, but now is %d'
                             % inputs.dim())
        drop = self.dropout_rate if (self.use_dropout and self.training) else 0.0
        seed = (self.seed * 1000003 + self._calls) & 0xFFFFFFFFFFFFFFFF
        self._calls += 1
        return _InteractingFn.apply(inputs.float(), self.kernel, self.bias, self.gamma, self.beta,
                                    self, seed, drop, lead.float(), grad_sink)


# ============================================================================================
# Dense / MultiLayerDense
# ============================================================================================
def _row_major(t: torch.Tensor) -> torch.Tensor:
    """A 2-D view the GEMM engine reads in place (unit column stride, any row stride >= width:
    a column slice of a concat buffer or of a split gradient); a copy only otherwise."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] and t.dtype == torch.float32:
        return t
    return t.contiguous().float()


class _GatherMultiFn(torch.autograd.Function):
    """outs[k][b, j] = src[b, plans[k][j]] (rs_gather_columns, one launch per plan); ONE backward
    for all of them: a zero-filled d_src and a scatter-add per plan (atomic adds: plans may
    overlap), instead of autograd's per-output zero fill + index_add + accumulate chain."""

    @staticmethod
    def forward(ctx, src, *plans):
        src = _row_major(src)
        B, S = src.shape
        outs = []
        for cols in plans:
            n = cols.numel()
            out = torch.empty(B, n, device=src.device, dtype=torch.float32)
            call("rs_gather_columns", stream_handle(), ptr(src), src.stride(0), B, ptr(cols), n,
                 ptr(out), n)
            outs.append(out)
        ctx.save_for_backward(*plans)
        ctx.shape = (B, S)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        plans = ctx.saved_tensors
        B, S = ctx.shape
        ref = next(d for d in douts if d is not None)
        dsrc = torch.zeros(B, S, device=ref.device, dtype=torch.float32)
        for cols, d in zip(plans, douts):
            if d is None:
                continue
            d = _row_major(d)
            call("rs_scatter_add_columns", stream_handle(), ptr(d), d.stride(0), B, ptr(cols),
                 cols.numel(), ptr(dsrc), S)
        return (dsrc,) + (None,) * len(plans)


def gather_multi(src, plans):
    """Column gathers of one [B, S] source (int32 column plans on the device)."""
    return _GatherMultiFn.apply(src, *plans)


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, act, sink=None):
        _lib.require_device(x, W)
        x = _row_major(x)
        M, K = x.shape
        N = W.shape[1]
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        call("rs_dense_fwd", stream_handle(), ptr(x), M, K, x.stride(0), ptr(W), ptr(b), N, act,
             ptr(y), N)
        ctx.save_for_backward(x, y, W, b)
        ctx.act = act
        ctx.sink = sink
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, W, b = ctx.saved_tensors
        dy = _row_major(dy)
        M, K = x.shape
        N = W.shape[1]
        s = stream_handle()
        ws_n = int(_lib.load().rs_dense_bwd_weight_workspace_floats(M, K, N))
        ws = torch.empty(ws_n, device=x.device, dtype=torch.float32)
        in_place = W.grad is not None and b.grad is not None and W.grad.is_contiguous()
        dW = W.grad if in_place else torch.empty_like(W)
        db = b.grad if in_place else torch.empty_like(b)
        dx = None
        sink = ctx.sink
        if ctx.needs_input_grad[0]:  # data and weight gradients in one launch
            if sink is not None and sink.buf is not None and tuple(sink.buf.shape) != (M, K):
                raise RuntimeError(f"GradSink holds a {tuple(sink.buf.shape)} gradient for a Dense "
                                   f"input of {(M, K)}: the producer's gradient would be lost")
            acc = sink is not None and sink.buf is not None
            dx = sink.buf if acc else torch.empty(M, K, device=x.device, dtype=torch.float32)
            if sink is not None:
                sink.buf = None
            call("rs_dense_bwd", s, ptr(x), x.stride(0), ptr(dy), dy.stride(0), ptr(y), N, ctx.act,
                 ptr(W), M, K, N, ptr(dx), K, 1 if acc else 0, ptr(dW), ptr(db),
                 1 if in_place else 0, ptr(ws), ws_n)
        else:
            call("rs_dense_bwd_weight", s, ptr(x), x.stride(0), ptr(dy), dy.stride(0), ptr(y), N,
                 ctx.act, M, K, N, ptr(dW), ptr(db), 1 if in_place else 0, ptr(ws), ws_n)
        if in_place:
            return dx, None, None, None, None
        return dx, dW, db, None, None


class Dense(nn.Module):
    """tf.keras.layers.Dense(units, activation): glorot_uniform kernel [in, units], zero bias."""

    def __init__(self, units, activation=None, seed=0, device=None, name=None):
        super().__init__()
        self.units = int(units)
        self.activation = activation
        self.act = _act_code(activation)
        self.seed = int(seed)
        self._device = device
        self.built = False
        self.name = name

    def build(self, input_shape, device=None):
        K = int(input_shape[-1])
        device = device or self._device or torch.device("cuda")
        blk = FlatBlock([(K, self.units), (self.units,)], device)
        self.kernel, self.bias = blk.params()
        glorot_uniform_(self.kernel, K, self.units, torch.Generator().manual_seed(self.seed))
        self.input_dim = K
        self.built = True

    def forward(self, x, grad_sink=None):
        """grad_sink: a GradSink whose producer's input gradient this layer's dx is added onto
        (see GradSink; only for a 2-D input)."""
        if not self.built:
            self.build(tuple(x.shape), device=x.device)
        lead = x.shape[:-1]  # Keras Dense = tensordot over the last axis
        from . import ops
        if ops.custom_ops_enabled():
            y = torch.ops.ctr.dense(x.reshape(-1, x.shape[-1]).float(), self.kernel, self.bias, self.act)
            return y.reshape(*lead, self.units)
        y = _DenseFn.apply(x.reshape(-1, x.shape[-1]).float(), self.kernel, self.bias, self.act,
                           grad_sink)
        return y.reshape(*lead, self.units)


def _desc_ptr(vals):
    """A host int64 descriptor array for the grouped Dense entries (kept alive by the caller)."""
    import ctypes
    arr = (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])
    return arr, ctypes.cast(arr, ctypes.c_void_p)


class _GroupedDenseFn(torch.autograd.Function):
    """G independent Dense layers in one forward launch and two (+ one reduce) backward launches
    (rs_dense_*_grouped).  apply(acts, x_0..x_{G-1}, W_0.., b_0..)."""

    @staticmethod
    def forward(ctx, acts, *t):
        G = len(acts)
        xs, Ws, bs = [_row_major(x) for x in t[:G]], t[G:2 * G], t[2 * G:]
        _lib.require_device(*xs, *Ws)
        ys, desc = [], []
        for x, W, b, a in zip(xs, Ws, bs, acts):
            M, K = x.shape
            N = W.shape[1]
            y = torch.empty(M, N, device=x.device, dtype=torch.float32)
            ys.append(y)
            desc += [M, K, N, x.stride(0), N, a, ptr(x), ptr(W), ptr(b), ptr(y)]
        keep, d = _desc_ptr(desc)
        call("rs_dense_fwd_grouped", stream_handle(), G, d)
        del keep
        ctx.save_for_backward(*xs, *ys, *Ws, *bs)
        ctx.acts = acts
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        acts = ctx.acts
        G = len(acts)
        sv = ctx.saved_tensors
        xs, ys, Ws, bs = sv[:G], sv[G:2 * G], sv[2 * G:3 * G], sv[3 * G:]
        dev = xs[0].device
        s = stream_handle()
        dys = [_row_major(d) if d is not None else torch.zeros_like(y) for d, y in zip(dys, ys)]
        dxs = [None] * G
        if any(ctx.needs_input_grad[1:1 + G]):
            desc = []
            for i in range(G):
                M, K = xs[i].shape
                N = Ws[i].shape[1]
                dxs[i] = torch.empty(M, K, device=dev, dtype=torch.float32)
                desc += [M, K, N, dys[i].stride(0), N, acts[i], ptr(dys[i]), ptr(ys[i]), ptr(Ws[i]),
                         ptr(dxs[i]), K, 0]
            keep, d = _desc_ptr(desc)
            call("rs_dense_bwd_data_grouped", s, G, d)
            del keep
        in_place = all(W.grad is not None and b.grad is not None and W.grad.is_contiguous()
                       for W, b in zip(Ws, bs))
        dWs = [W.grad if in_place else torch.empty_like(W) for W in Ws]
        dbs = [b.grad if in_place else torch.empty_like(b) for b in bs]
        desc = []
        for i in range(G):
            M, K = xs[i].shape
            N = Ws[i].shape[1]
            desc += [M, K, N, xs[i].stride(0), dys[i].stride(0), N, acts[i], ptr(xs[i]), ptr(dys[i]),
                     ptr(ys[i]), ptr(dWs[i]), ptr(dbs[i]), 1 if in_place else 0]
        keep, d = _desc_ptr(desc)
        ws_n = int(_lib.load().rs_dense_bwd_weight_grouped_workspace_floats(G, d))
        ws = torch.empty(max(ws_n, 1), device=dev, dtype=torch.float32)
        call("rs_dense_bwd_weight_grouped", s, G, d, ptr(ws), ws_n)
        del keep
        if in_place:
            return (None, *dxs) + (None,) * (2 * G)
        return (None, *dxs, *dWs, *dbs)


def grouped_dense(layers, xs):
    """[layer_i(x_i)] for built Dense layers of one input rank, as ONE grouped launch per pass
    (same math as calling each layer; the per-expert / per-task loops of staytime/VideoDnn.py and
    rough_rank/layer.py).  Up to 8 layers per group."""
    layers, xs = list(layers), list(xs)
    if len(layers) == 1 or len(layers) > 8:
        return [l(x) for l, x in zip(layers, xs)]
    for l, x in zip(layers, xs):
        if not l.built:
            l.build(tuple(x.shape), device=x.device)
    acts = tuple(l.act for l in layers)
    flat = [x.reshape(-1, x.shape[-1]).float() for x in xs]
    ys = _GroupedDenseFn.apply(acts, *flat, *[l.kernel for l in layers], *[l.bias for l in layers])
    return [y.reshape(*x.shape[:-1], l.units) for y, x, l in zip(ys, xs, layers)]


class MultiLayerDense(nn.Module):
    """MultiLayerDense(units=[...], activation=...) (imported at autoint:9, absent from the
    reference): pinned as Dense(u, activation) for every u in order."""

    def __init__(self, units, activation="relu", seed=0, device=None):
        super().__init__()
        self.units = [int(u) for u in units]
        self.activation = activation
        self.layers = nn.ModuleList(
            Dense(u, activation, seed=seed + i, device=device) for i, u in enumerate(self.units))

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x
