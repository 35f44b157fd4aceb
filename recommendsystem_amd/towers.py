"""Tower layers of the ranking models, keeping the reference's Keras
constructor kwargs and call signatures; compute runs in librecsys_amd.so (csrc/dense.hip for the
GEMMs, csrc/towers.hip for everything around them).

    DNN, MMOE, PLE, CrossNet, KDLoss, Similarity      rough_rank/layer.py
    DeepCrossLayer, FMLayer                           staytime/layer.py:44-116
    SENetFM, FFMBlock, PPNetGate, StaytimeHead        staytime/VideoDnn.py:11-25,81-179
    keras_bce, custom_kl_loss                         rough_rank/model.py:211-214, staytime/model.py:20-30

MI355X shape of the mixture layers: every expert's first Dense and every task gate read the
same input, so MMOE / PLE keep their kernels as column blocks of ONE [K, sum N] matrix: one
MFMA GEMM produces all expert pre-activations and gate logits, and one rs_gate_mix pass applies
the expert activation, the gate softmax and the weighted sum (and the reverse in backward).
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle
from .layers import Dense, _act_code, _DenseFn, _row_major
from .params import FlatBlock, glorot_uniform_, grads_contiguous


def glorot_normal_(t: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator | None) -> None:
    """Keras GlorotNormal: truncated normal (2 sigma), stddev sqrt(2/(in+out)) / .87962566."""
    std = math.sqrt(2.0 / float(fan_in + fan_out)) / 0.87962566103423978
    with torch.no_grad():
        v = torch.randn(t.shape, generator=gen, dtype=torch.float64)
        bad = v.abs() > 2.0
        while bool(bad.any()):
            v[bad] = torch.randn(int(bad.sum()), generator=gen, dtype=torch.float64)
            bad = v.abs() > 2.0
        t.copy_(v * std)


def _rows(x: torch.Tensor) -> torch.Tensor:
    """2-D fp32 view with unit column stride (copy only if needed)."""
    x = x.float()
    if x.dim() != 2 or x.stride(-1) != 1:
        x = x.reshape(-1, x.shape[-1]).contiguous()
    return x


def _split_grads(params, dparams):
    outs, off = [], 0
    for p in params:
        outs.append(dparams[off:off + p.numel()].view(p.shape))
        off += p.numel()
    return outs


# ============================================================================================
# DNN (rough_rank/layer.py:33-117)
# ============================================================================================
class DNN(nn.Module):
    """DNN(hidden_units, activation='relu', l2_reg=0, dropout_rate=0, use_bn=False,
    output_activation=None, seed=None): GlorotNormal kernels, zero biases, Activation after each
    layer (output_activation on the last when given).  BatchNormalization / dropout are not on
    the path (every call site uses use_bn=False, dropout_rate=0) and raise NotImplementedError.
    l2_reg is a loss-side regulariser: ``regularization_loss()`` returns l2_reg * sum ||W||^2."""

    def __init__(self, hidden_units, activation="relu", l2_reg=0, dropout_rate=0, use_bn=False,
                 output_activation=None, seed=None, device=None, **kwargs):
        super().__init__()
        if use_bn or dropout_rate:
            raise NotImplementedError("DNN with use_bn / dropout is not on the fused path")
        self.hidden_units = [int(u) for u in hidden_units]
        self.activation = activation
        self.output_activation = output_activation
        self.l2_reg = float(l2_reg)
        self.seed = 0 if seed is None else int(seed)
        self.name = kwargs.get("name", "dnn")
        n = len(self.hidden_units)
        acts = [activation] * n
        if n and output_activation:
            acts[-1] = output_activation
        acts = [None if a == "linear" else a for a in acts]
        self.layers = nn.ModuleList(Dense(u, a, seed=self.seed + i, device=device)
                                    for i, (u, a) in enumerate(zip(self.hidden_units, acts)))
        self._device = device
        self.built = False

    def build(self, input_shape, device=None):
        K = int(input_shape[-1])
        gen = torch.Generator().manual_seed(self.seed)
        for layer in self.layers:
            layer.build((None, K), device=device or self._device)
            glorot_normal_(layer.kernel, K, layer.units, gen)
            K = layer.units
        self.built = True

    def forward(self, x):
        if not self.built:
            self.build(tuple(x.shape), device=x.device)
        for layer in self.layers:
            x = layer(x)
        return x

    def regularization_loss(self):
        return self.l2_reg * sum(torch.sum(l.kernel * l.kernel) for l in self.layers)


# ============================================================================================
# Expert / gate mixture (MMOE, PLE, multi_head gates)
# ============================================================================================
class _MixFn(torch.autograd.Function):
    """Z [M, n_exp*D + n_task*n_sel] (expert pre-activations, then gate logits) -> [M, n_task*D]."""

    @staticmethod
    def forward(ctx, Z, sel, n_exp, D, n_task, n_sel, e_act):
        M = Z.shape[0]
        Y = torch.empty(M, n_task * D, device=Z.device, dtype=torch.float32)
        goff = n_exp * D
        call("rs_gate_mix_fwd", stream_handle(), ptr(Z), Z.stride(0), e_act, Z.data_ptr() + 4 * goff,
             Z.stride(0), M, n_exp, D, n_task, n_sel, ptr(sel), ptr(Y), n_task * D, None, 0)
        ctx.save_for_backward(Z, sel)
        ctx.cfg = (n_exp, D, n_task, n_sel, e_act)
        return Y

    @staticmethod
    def backward(ctx, dY):
        Z, sel = ctx.saved_tensors
        n_exp, D, n_task, n_sel, e_act = ctx.cfg
        dY = dY.contiguous()
        M = Z.shape[0]
        dZ = torch.empty_like(Z)
        goff = n_exp * D
        call("rs_gate_mix_bwd", stream_handle(), ptr(Z), Z.stride(0), e_act, Z.data_ptr() + 4 * goff,
             Z.stride(0), M, n_exp, D, n_task, n_sel, ptr(sel), ptr(dY), n_task * D, ptr(dZ),
             dZ.stride(0), dZ.data_ptr() + 4 * goff, dZ.stride(0))
        return dZ, None, None, None, None, None, None


class ExpertGateLayer(nn.Module):
    """n_exp single-Dense experts (width D, activation e_act) and n_task softmax gates over
    n_sel selected experts, all reading the same input: one concatenated [K, n_exp*D +
    n_task*n_sel] kernel (column blocks = the Keras layers' kernels) -> rs_gate_mix.
    ``sel[t]`` lists the experts task t mixes (MMOE: all; PLE: shared + its own)."""

    def __init__(self, n_exp, D, sel: Sequence[Sequence[int]], expert_activation="relu",
                 expert_init="glorot_normal", gate_init="glorot_normal", seed=0, device=None):
        super().__init__()
        self.n_exp, self.D = int(n_exp), int(D)
        self.sel_list = [list(map(int, s)) for s in sel]
        self.n_task = len(self.sel_list)
        self.n_sel = len(self.sel_list[0])
        if any(len(s) != self.n_sel for s in self.sel_list):
            raise ValueError("every task must mix the same number of experts")
        self.e_act = _act_code(expert_activation)
        self.expert_init, self.gate_init = expert_init, gate_init
        self.seed = int(seed)
        self._device = device
        self.built = False

    @property
    def n_cols(self):
        return self.n_exp * self.D + self.n_task * self.n_sel

    def build(self, input_shape, device=None):
        K = int(input_shape[-1])
        device = device or self._device or torch.device("cuda")
        blk = FlatBlock([(K, self.n_cols), (self.n_cols,)], device)
        self.kernel, self.bias = blk.params()
        gen = torch.Generator().manual_seed(self.seed)
        for e in range(self.n_exp):
            self._init(self.expert_kernel(e), K, self.D, self.expert_init, gen)
        for t in range(self.n_task):
            self._init(self.gate_kernel(t), K, self.n_sel, self.gate_init, gen)
        self.sel = torch.tensor(self.sel_list, dtype=torch.int32, device=device).reshape(-1)
        self.input_dim = K
        self.built = True

    @staticmethod
    def _init(view, fan_in, fan_out, kind, gen):
        t = torch.empty(view.shape)
        if kind == "glorot_normal":
            glorot_normal_(t, fan_in, fan_out, gen)
        elif kind == "glorot_uniform":
            glorot_uniform_(t, fan_in, fan_out, gen)
        elif isinstance(kind, tuple) and kind[0] == "truncated_normal":  # TruncatedNormal(stddev)
            v = torch.randn(t.shape, generator=gen, dtype=torch.float64)
            v = torch.where(v.abs() > 2, torch.randn(t.shape, generator=gen, dtype=torch.float64), v)
            t.copy_(v.clamp(-2, 2) * kind[1])
        with torch.no_grad():
            view.copy_(t)

    # Keras-layer views of the concatenated kernel
    def expert_kernel(self, e):
        return self.kernel[:, e * self.D:(e + 1) * self.D]

    def expert_bias(self, e):
        return self.bias[e * self.D:(e + 1) * self.D]

    def gate_kernel(self, t):
        o = self.n_exp * self.D + t * self.n_sel
        return self.kernel[:, o:o + self.n_sel]

    def gate_bias(self, t):
        o = self.n_exp * self.D + t * self.n_sel
        return self.bias[o:o + self.n_sel]

    def forward_flat(self, x):
        """All task outputs side by side, [B, n_task * D] (= torch.cat(forward(x), 1)): consumers
        that concatenate the task outputs anyway take this and skip the per-slice backward
        (7 zero-fills + copies + adds per step at config 3)."""
        if not self.built:
            self.build(tuple(x.shape), device=x.device)
        x = _rows(x)
        Z = _DenseFn.apply(x, self.kernel, self.bias, 0)
        return _MixFn.apply(Z, self.sel, self.n_exp, self.D, self.n_task, self.n_sel, self.e_act)

    def forward(self, x):
        Y = self.forward_flat(x)
        return [Y[:, t * self.D:(t + 1) * self.D] for t in range(self.n_task)]


def _single_layer(units, params, gate_units):
    if len(units) != 1 or list(gate_units):
        raise NotImplementedError("MMOE/PLE with multi-layer experts or gate hidden layers is not "
                                  "on the fused path (every call site uses one expert layer and "
                                  "gate_dnn_units=())")
    params = dict(params or {})
    act = params.pop("activation", "relu")
    for k in ("l2_reg", "dropout_rate", "use_bn", "seed", "output_activation"):
        params.pop(k, None)
    if params:
        raise NotImplementedError(f"unsupported DNN params {sorted(params)}")
    return int(units[0]), act


class MMOE(nn.Module):
    """MMOE(num_tasks, num_experts=2, expert_dnn_units=(32,), gate_dnn_units=(),
    expert_dnn_params=None, gate_dnn_params=None) (rough_rank/layer.py:120-171) -> list of
    num_tasks [B, expert_dim] task outputs."""

    def __init__(self, num_tasks, num_experts=2, expert_dnn_units=(32,), gate_dnn_units=(),
                 expert_dnn_params=None, gate_dnn_params=None, seed=0, device=None, **kwargs):
        super().__init__()
        D, act = _single_layer(expert_dnn_units, expert_dnn_params, gate_dnn_units)
        self.num_tasks, self.num_experts = int(num_tasks), int(num_experts)
        sel = [list(range(self.num_experts)) for _ in range(self.num_tasks)]
        self.mix = ExpertGateLayer(self.num_experts, D, sel, act, seed=seed, device=device)
        self.name = kwargs.get("name", "mmoe")

    def forward(self, inputs):
        return self.mix(inputs)


class PLE(nn.Module):
    """PLE(num_tasks, num_shared_experts=2, num_specific_experts=2, expert_dnn_units=(32,),
    gate_dnn_units=(), ...) (rough_rank/layer.py:174-233).  Expert order in the concatenated
    kernel: shared 0..S-1, then task t's specific experts; task t mixes [shared, its own]."""

    def __init__(self, num_tasks, num_shared_experts=2, num_specific_experts=2,
                 expert_dnn_units=(32,), gate_dnn_units=(), expert_dnn_params=None,
                 gate_dnn_params=None, seed=0, device=None, **kwargs):
        super().__init__()
        D, act = _single_layer(expert_dnn_units, expert_dnn_params, gate_dnn_units)
        T, S, P = int(num_tasks), int(num_shared_experts), int(num_specific_experts)
        self.num_tasks, self.num_shared_experts, self.num_specific_experts = T, S, P
        sel = [list(range(S)) + [S + t * P + j for j in range(P)] for t in range(T)]
        self.mix = ExpertGateLayer(S + T * P, D, sel, act, seed=seed, device=device)
        self.name = kwargs.get("name", "ple")

    def forward(self, inputs):
        return self.mix(inputs)


# ============================================================================================
# CrossNet / DeepCrossLayer
# ============================================================================================
class _CrossFn(torch.autograd.Function):
    """lead [M, Dl] (optional): return the concat [lead, y] [M, Dl + D] with y written in place by
    the kernel (ldy) and its gradient read from the concat's slice (lddy) -- no concat copy."""

    @staticmethod
    def forward(ctx, x, W, b, L, lead=None):
        _lib.require_device(x, W)
        x = _rows(x)
        M, D = x.shape
        Dl = 0 if lead is None else lead.shape[1]
        out = torch.empty(M, Dl + D, device=x.device, dtype=torch.float32)
        if lead is not None:
            out[:, :Dl].copy_(lead)
        call("rs_cross_fwd", stream_handle(), ptr(x), x.stride(0), M, D, L, ptr(W), ptr(b),
             out.data_ptr() + 4 * Dl, Dl + D)
        ctx.save_for_backward(x, W, b)
        ctx.L, ctx.Dl = L, Dl
        return out

    @staticmethod
    def backward(ctx, dout):
        x, W, b = ctx.saved_tensors
        L, Dl = ctx.L, ctx.Dl
        dout = _row_major(dout)
        d_lead = dout[:, :Dl] if Dl else None
        dy = dout[:, Dl:] if Dl else dout
        M, D = x.shape
        dx = torch.empty(M, D, device=x.device, dtype=torch.float32)
        ws_n = int(_lib.load().rs_cross_bwd_workspace_floats(M, D, L))
        ws = torch.empty(max(ws_n, 1), device=x.device, dtype=torch.float32)
        block = grads_contiguous((W, b))
        dpar = block if block is not None else torch.empty(2 * L * D, device=x.device)
        call("rs_cross_bwd", stream_handle(), ptr(x), x.stride(0), M, D, L, ptr(W), ptr(b), ptr(dy),
             dy.stride(0), ptr(dx), D, 0, ptr(dpar), 1 if block is not None else 0, ptr(ws), ws_n)
        if block is not None:
            return dx, None, None, None, d_lead
        dW, db = _split_grads((W, b), dpar)
        return dx, dW, db, None, d_lead


class _CrossBase(nn.Module):
    def __init__(self, layer_num, init, seed, device):
        super().__init__()
        self.layer_num = int(layer_num)
        self._init, self.seed, self._device = init, seed, device
        self.built = False

    def build(self, input_shape, device=None):
        D = int(input_shape[-1])
        device = device or self._device or torch.device("cuda")
        blk = FlatBlock([(self.layer_num, D), (self.layer_num, D)], device)
        self.W, self.b = blk.params()
        gen = torch.Generator().manual_seed(self.seed)
        for l in range(self.layer_num):  # each kernel is a [D, 1] Keras weight
            t = torch.empty(D, 1)
            (glorot_normal_ if self._init == "glorot_normal" else glorot_uniform_)(t, D, 1, gen)
            with torch.no_grad():
                self.W[l].copy_(t[:, 0])
        self.input_dim = D
        self.built = True

    def forward(self, inputs):
        if inputs.dim() != 2:
            raise ValueError("cross layers take a 2-D input [batch, dim]")
        if not self.built:
            self.build(tuple(inputs.shape), device=inputs.device)
        return _CrossFn.apply(inputs, self.W, self.b, self.layer_num)

    def forward_concat(self, lead, inputs):
        """torch.cat([lead, self(inputs)], dim=1) with the cross output written into the concat
        (staytime/VideoDnn.py:168 ext = concat([mmoe[0], cross]))."""
        if inputs.dim() != 2 or lead.dim() != 2:
            raise ValueError("cross layers take 2-D inputs [batch, dim]")
        if not self.built:
            self.build(tuple(inputs.shape), device=inputs.device)
        return _CrossFn.apply(inputs, self.W, self.b, self.layer_num, lead.float())


class CrossNet(_CrossBase):
    """CrossNet(layer_num=2, l2_reg=0, seed=1024) (rough_rank/layer.py:236-270): kernels [D, 1]
    GlorotNormal, biases [D, 1] zeros, x_{l+1} = x0 (x_l . w_l) + b_l + x_l."""

    def __init__(self, layer_num=2, l2_reg=0, seed=1024, device=None, **kwargs):
        super().__init__(layer_num, "glorot_normal", seed, device)
        self.l2_reg = float(l2_reg)


class DeepCrossLayer(_CrossBase):
    """DeepCrossLayer(num_layer=3) (staytime/layer.py:44-80): W_i [D, 1] glorot_uniform, b_i [D]
    zeros; the same recurrence (cross_0 uses the input for both x0 and x_l)."""

    def __init__(self, num_layer=3, seed=0, device=None, **kwargs):
        super().__init__(num_layer, "glorot_uniform", seed, device)
        self.num_layer = self.layer_num


# ============================================================================================
# FM family
# ============================================================================================
class _FMFn(torch.autograd.Function):
    """x [M, F, E] (any strides with unit e-stride), optional scale a [M, F] ->
    (y = x * a [M, F*E] or None, cross [M, E], fm [M, 1])."""

    @staticmethod
    def forward(ctx, x, a, want_y, a_scale=1.0):
        M, F, E = x.shape
        if x.stride(2) != 1 or x.stride(1) < E:
            x = x.contiguous()
        dev = x.device
        y = torch.empty(M, F * E, device=dev) if want_y else None
        c = torch.empty(M, E, device=dev)
        fm = torch.empty(M, 1, device=dev)
        a_ = a.contiguous() if a is not None else None
        call("rs_fm_fwd", stream_handle(), ptr(x), x.stride(0), x.stride(1), M, F, E, ptr(a_),
             F if a_ is not None else 0, a_scale, ptr(y), F * E, ptr(c), E, ptr(fm), 1)
        ctx.save_for_backward(x, a_)
        ctx.want_y, ctx.a_scale = want_y, a_scale
        return (y if want_y else c.new_empty(0)), c, fm

    @staticmethod
    def backward(ctx, dy, dc, dfm):
        x, a = ctx.saved_tensors
        M, F, E = x.shape
        dev = x.device
        dx = torch.empty(M, F, E, device=dev)
        da = torch.empty(M, F, device=dev) if (a is not None and ctx.needs_input_grad[1]) else None
        # column slices of a concat gradient are read in place (row strides), not copied
        dy = _row_major(dy) if (ctx.want_y and dy is not None and dy.numel()) else None
        dc = _row_major(dc) if dc is not None else None
        dfm = _row_major(dfm) if dfm is not None else None
        call("rs_fm_bwd", stream_handle(), ptr(x), x.stride(0), x.stride(1), M, F, E, ptr(a),
             F if a is not None else 0, ctx.a_scale, ptr(dy), dy.stride(0) if dy is not None else 0,
             ptr(dc), dc.stride(0) if dc is not None else 0, ptr(dfm),
             dfm.stride(0) if dfm is not None else 1, ptr(dx), F * E, E, 0, ptr(da), F)
        return dx, da, None, None


class FMLayer(nn.Module):
    """FMLayer() (staytime/layer.py:83-116, rank/finish/videodnn.py:23-52): [B, F, E] -> [B, 1]
    = 0.5 sum_e ((sum_f x)^2 - sum_f x^2)."""

    def forward(self, inputs):
        if inputs.dim() != 3:
            raise ValueError("Unexpected inputs dimensions %d, expect to be 3 dimensions" % inputs.dim())
        _, _, fm = _FMFn.apply(inputs.float(), None, False)
        return fm


class SENetFM(nn.Module):
    """staytime/VideoDnn.py:81-115: SENet squeeze (Dense(int(F/4), relu) on the stop-gradient
    concat of the F general inputs), excite 2 * Dense(F, sigmoid), per-field reweight, FM cross
    term and fm_logit.  Input x [B, F, E] (e.g. the [:, :, 0:16] slice of the lookup).
    Returns (reweighted [B, F*E], cross_term [B, E], fm_logit [B, 1])."""

    def __init__(self, num_fields, seed=0, device=None):
        super().__init__()
        F = int(num_fields)
        self.num_fields = F
        # senet_unit1 = len / 4 is a float; Keras Dense coerces units with int() (pinned)
        self.squeeze = Dense(int(F / 4), "relu", seed=seed, device=device, name="senet_squeeze_layer1")
        self.excite = Dense(F, "sigmoid", seed=seed + 1, device=device, name="senet_extract_layer2")
        self._two = None

    def forward(self, x):
        B, F, E = x.shape
        sq = x.detach().reshape(B, F * E)             # tf.stop_gradient(concat(general_inputs))
        s1 = self.squeeze(sq)
        s2 = self.excite(s1)                       # sigmoid; the factor 2 is the FM kernel's a_scale
        y, cross, fm = _FMFn.apply(x, s2, True, 2.0)
        return y, cross, fm


class _FFMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Wx, bx, Wy, by, cols, NU, NI, Dff, with_mult):
        M = x.shape[0]
        dev = x.device
        P = NU * NI
        y = torch.empty(M, P * Dff, device=dev)
        mu = torch.empty(M, NU * 16, device=dev) if with_mult else None
        call("rs_ffm_fwd", stream_handle(), ptr(x), x.stride(0), M, NU, NI, 16, Dff, ptr(cols), ptr(Wx),
             ptr(bx), ptr(Wy), ptr(by), ptr(y), P * Dff, ptr(mu), NU * 16)
        ctx.save_for_backward(x, Wx, bx, Wy, by, cols)
        ctx.cfg = (NU, NI, Dff, with_mult)
        return y, (mu if with_mult else y.new_empty(0))

    @staticmethod
    def backward(ctx, dy, dmu):
        x, Wx, bx, Wy, by, cols = ctx.saved_tensors
        NU, NI, Dff, with_mult = ctx.cfg
        M = x.shape[0]
        dy = _row_major(dy)
        dmu = _row_major(dmu) if (with_mult and dmu is not None and dmu.numel()) else None
        dx = torch.zeros_like(x)
        lib = _lib.load()
        ws_n = int(lib.rs_ffm_bwd_workspace_floats(M, NU, NI, 16, Dff))
        ws = torch.empty(max(ws_n, 1), device=x.device)
        params = (Wx, bx, Wy, by)
        block = grads_contiguous(params)
        dpar = block if block is not None else torch.empty(sum(p.numel() for p in params), device=x.device)
        call("rs_ffm_bwd", stream_handle(), ptr(x), x.stride(0), M, NU, NI, 16, Dff, ptr(cols), ptr(Wx),
             ptr(bx), ptr(Wy), ptr(by), ptr(dy), dy.stride(0), ptr(dmu),
             dmu.stride(0) if dmu is not None else NU * 16, ptr(dx),
             x.stride(0), 1, ptr(dpar), 1 if block is not None else 0, ptr(ws), ws_n)
        g = (None,) * 4 if block is not None else tuple(_split_grads(params, dpar))
        return (dx, *g, None, None, None, None, None)


class FFMBlock(nn.Module):
    """ffm_block(slot_dict, [[x_list, y_list, dim]]) (staytime/VideoDnn.py:11-25) + the
    user x item multiply-ReLU (:99-105), fused.  Input: x [B, F*16] (the general inputs, field k
    at columns k*16 .. k*16+15) and the user / item field indices.  Pair p = (i, j) owns
    Dense(dim) 'ffm_x_*' on x_i and 'ffm_y_*' on y_j (glorot_uniform, zero bias).
    Returns (ffm [B, NU*NI*dim], multiply [B, NU*16] or None)."""

    def __init__(self, user_fields, item_fields, dim=8, with_multiply=True, seed=0, device=None,
                 field_stride=16):
        super().__init__()
        self.user_fields, self.item_fields = list(user_fields), list(item_fields)
        self.NU, self.NI, self.dim = len(self.user_fields), len(self.item_fields), int(dim)
        self.with_multiply = bool(with_multiply)
        device = device or torch.device("cuda")
        P, E = self.NU * self.NI, 16
        blk = FlatBlock([(P, E, self.dim), (P, self.dim), (P, E, self.dim), (P, self.dim)], device)
        self.Wx, self.bx, self.Wy, self.by = blk.params()
        gen = torch.Generator().manual_seed(seed)
        for p in range(P):
            for W in (self.Wx, self.Wy):
                t = torch.empty(E, self.dim)
                glorot_uniform_(t, E, self.dim, gen)
                with torch.no_grad():
                    W[p].copy_(t)
        self.cols = torch.tensor([f * int(field_stride) for f in self.user_fields + self.item_fields],
                                 dtype=torch.int32, device=device)

    def forward(self, x):
        x = _rows(x)  # [B, fields * field_stride]; field k's 16 columns start at k * field_stride
        y, mu = _FFMFn.apply(x, self.Wx, self.bx, self.Wy, self.by, self.cols, self.NU, self.NI,
                             self.dim, self.with_multiply)
        return y, (mu if self.with_multiply else None)


class _MulFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, g, scale):
        a, g = _rows(a), _rows(g)
        M, N = a.shape
        y = torch.empty(M, N, device=a.device)
        call("rs_mul_fwd", stream_handle(), ptr(a), a.stride(0), ptr(g), g.stride(0), M, N, scale,
             ptr(y), N)
        ctx.save_for_backward(a, g)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        a, g = ctx.saved_tensors
        M, N = a.shape
        dy = _row_major(dy)
        da = torch.empty(M, N, device=a.device, dtype=torch.float32)
        dg = torch.empty(M, N, device=a.device, dtype=torch.float32)
        call("rs_mul_bwd", stream_handle(), ptr(a), a.stride(0), ptr(g), g.stride(0), M, N, ctx.scale,
             ptr(dy), dy.stride(0), ptr(da), N, ptr(dg), N)
        return da, dg, None


class _GroupedMulFn(torch.autograd.Function):
    """Y_i = A_i * (scale G_i) for G <= 8 pairs in one launch each way (rs_mul_*_grouped)."""

    @staticmethod
    def forward(ctx, scale, *t):
        from .layers import _desc_ptr
        G = len(t) // 2
        As, Gs = [_rows(a) for a in t[:G]], [_rows(g) for g in t[G:]]
        ys, desc = [], []
        for a, g in zip(As, Gs):
            M, N = a.shape
            y = torch.empty(M, N, device=a.device)
            ys.append(y)
            desc += [M, N, a.stride(0), g.stride(0), N, ptr(a), ptr(g), ptr(y)]
        keep, d = _desc_ptr(desc)
        call("rs_mul_fwd_grouped", stream_handle(), G, d, float(scale))
        del keep
        ctx.save_for_backward(*As, *Gs)
        ctx.scale = float(scale)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        from .layers import _desc_ptr
        sv = ctx.saved_tensors
        G = len(sv) // 2
        As, Gs = sv[:G], sv[G:]
        das, dgs, desc = [], [], []
        for a, g, dy in zip(As, Gs, dys):
            M, N = a.shape
            dy = _row_major(dy) if dy is not None else torch.zeros(M, N, device=a.device)
            da = torch.empty(M, N, device=a.device)
            dg = torch.empty(M, N, device=a.device)
            das.append(da)
            dgs.append(dg)
            desc += [M, N, a.stride(0), g.stride(0), dy.stride(0), N, N, ptr(a), ptr(g), ptr(dy),
                     ptr(da), ptr(dg)]
        keep, d = _desc_ptr(desc)
        call("rs_mul_bwd_grouped", stream_handle(), G, d, ctx.scale)
        del keep
        return (None, *das, *dgs)


def gated_group(deeps, gates, scale=2.0):
    """[gated(d, g, scale)] for up to 8 (deep, gate) pairs in one launch per pass."""
    if len(deeps) == 1 or len(deeps) > 8:
        return [gated(d, g, scale) for d, g in zip(deeps, gates)]
    return list(_GroupedMulFn.apply(float(scale), *deeps, *gates))


def gated(deep, gate, scale=2.0):
    """ppnet gating tf.multiply(2 * sigmoid_gate, deep) (staytime/VideoDnn.py:139-146)."""
    return _MulFn.apply(deep, gate, float(scale))


class PPNetExperts(nn.Module):
    """The ppnet-gated expert stacks of staytime/VideoDnn.py:129-148: expert i, layer j:
    gate = 2 * Dense(u, sigmoid)(Dense(u, relu)(gate_input)); deep = Dense(u, relu)(deep) * gate.
    Returns the stacked expert outputs [B, num_experts * units[-1]] (expert-major), the layout
    rs_gate_mix reads."""

    def __init__(self, num_experts, hidden_units, seed=0, device=None):
        super().__init__()
        self.num_experts, self.units = int(num_experts), [int(u) for u in hidden_units]
        mk = lambda u, a, s: Dense(u, a, seed=s, device=device)  # noqa: E731
        self.gate1 = nn.ModuleList(nn.ModuleList(mk(u, "relu", seed + 100 * i + 3 * j) for j, u in enumerate(self.units)) for i in range(self.num_experts))
        self.gate2 = nn.ModuleList(nn.ModuleList(mk(u, "sigmoid", seed + 100 * i + 3 * j + 1) for j, u in enumerate(self.units)) for i in range(self.num_experts))
        self.expert = nn.ModuleList(nn.ModuleList(mk(u, "relu", seed + 100 * i + 3 * j + 2) for j, u in enumerate(self.units)) for i in range(self.num_experts))

    def forward(self, concated_input, gate_input):
        outs = []
        for i in range(self.num_experts):
            deep = concated_input
            for j in range(len(self.units)):
                g = self.gate2[i][j](self.gate1[i][j](gate_input))
                deep = gated(self.expert[i][j](deep), g, 2.0)
            outs.append(deep)
        return outs


# ============================================================================================
# heads and losses
# ============================================================================================
class _SoftmaxKLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y_true, sample_w, bins, loss_weight):
        z = _rows(z)
        M, C = z.shape
        dev = z.device
        P = torch.empty(M, C + 1, device=dev)
        rows = torch.empty(M, device=dev)
        dz = torch.empty(M, C, device=dev)
        yt = _rows(y_true)
        sw = sample_w.reshape(-1).float().contiguous() if sample_w is not None else None
        # gscale folds the Keras reduction (sum over the batch / batch size) and the loss weight
        call("rs_softmax_kl", stream_handle(), ptr(z), z.stride(0), M, C, ptr(bins), ptr(P), C + 1,
             ptr(yt), yt.stride(0), ptr(sw), float(loss_weight) / M, 1e-7, ptr(rows), ptr(dz), C)
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(P)
        ctx.set_materialize_grads(False)  # no zero-filled grad for P
        return rows.sum() * (float(loss_weight) / M), P

    @staticmethod
    def backward(ctx, dloss, _dP):
        (dz,) = ctx.saved_tensors
        return dz * dloss, None, None, None, None


class StaytimeHead(nn.Module):
    """staytime/VideoDnn.py:168-179 + custom_kl_loss (staytime/model.py:20-30): Dense(400) over
    [mmoe_out, cross], softmax, expected watch time over the bins (clamped at 0).  ``forward``
    returns final_y_pred [B, 401]; ``loss`` returns (weighted KL loss, final_y_pred) with the
    softmax + KL gradient fused into one kernel."""

    def __init__(self, bins: Sequence[float], seed=0, device=None):
        super().__init__()
        self.C = len(bins)
        self.dense = Dense(self.C, None, seed=seed, device=device, name="staytime_output")
        self._bins_list = [float(b) for b in bins]
        self.bins = None

    def _bins(self, dev):
        if self.bins is None or self.bins.device != dev:
            self.bins = torch.tensor(self._bins_list, dtype=torch.float32, device=dev)
        return self.bins

    def forward(self, x):
        z = _rows(self.dense(x))
        M = z.shape[0]
        P = torch.empty(M, self.C + 1, device=z.device)
        call("rs_softmax_kl", stream_handle(), ptr(z), z.stride(0), M, self.C, ptr(self._bins(z.device)),
             ptr(P), self.C + 1, None, 0, None, 0.0, 1e-7, None, None, 0)
        return P

    def loss(self, x, y_true, sample_weight=None, loss_weight=1.0):
        z = self.dense(x)
        return _SoftmaxKLFn.apply(z, y_true, sample_weight, self._bins(z.device), loss_weight)

    def loss_term(self, x, y_true, sample_weight=None, loss_weight=1.0):
        """(LossTerm of custom_kl_loss for fused_loss, final_y_pred [B, 401]); P is written by
        the term's launch (softmax, expected watch time and the KL rows + dZ: one kernel)."""
        z = _rows(self.dense(x))
        M, C = z.shape
        P = torch.empty(M, C + 1, device=z.device)
        yt = _rows(y_true)
        sw = sample_weight.reshape(-1).float().contiguous() if sample_weight is not None else None
        bins = self._bins(z.device)

        def launch(rows, grad, gscale):
            call("rs_softmax_kl", stream_handle(), ptr(z), z.stride(0), M, C, ptr(bins), ptr(P), C + 1,
                 ptr(yt), yt.stride(0), ptr(sw), gscale, 1e-7, ptr(rows), ptr(grad), C)
        return LossTerm(z, loss_weight, launch), P


class _RowDotFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, v, sig):
        u, v = _rows(u), _rows(v)
        M, N = u.shape
        y = torch.empty(M, 1, device=u.device)
        call("rs_rowdot", stream_handle(), ptr(u), u.stride(0), ptr(v), v.stride(0), M, N, int(sig),
             ptr(y), None, None, 0, None, 0)
        ctx.save_for_backward(u, v)
        ctx.sig = sig
        return y

    @staticmethod
    def backward(ctx, dy):
        u, v = ctx.saved_tensors
        M, N = u.shape
        du, dv = torch.empty_like(u), torch.empty_like(v)
        call("rs_rowdot", stream_handle(), ptr(u), u.stride(0), ptr(v), v.stride(0), M, N,
             int(ctx.sig), None, ptr(dy.contiguous()), ptr(du), N, ptr(dv), N)
        return du, dv, None


class Similarity(nn.Module):
    """Similarity(use_sigmoid=False)([user_emb, item_emb]) (rough_rank/layer.py:6-30)."""

    def __init__(self, use_sigmoid=False, **kwargs):
        super().__init__()
        self.use_sigmoid = bool(use_sigmoid)

    def forward(self, inputs):
        u, i = inputs
        return _RowDotFn.apply(u, i, self.use_sigmoid)


class _MSERowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t):
        s, t = _rows(s), _rows(t)
        M, N = s.shape
        rows = torch.empty(M, device=s.device)
        call("rs_mse_rows", stream_handle(), ptr(s), s.stride(0), ptr(t), t.stride(0), M, N, 1.0,
             ptr(rows), None, 0)
        ctx.save_for_backward(s, t)
        return rows

    @staticmethod
    def backward(ctx, drows):
        s, t = ctx.saved_tensors
        M, N = s.shape
        # d/ds of mean_j (s - t)^2 per row, scaled by the incoming row gradients
        ds = dt = None
        if ctx.needs_input_grad[0]:
            ds = torch.empty_like(s)
            call("rs_mse_rows", stream_handle(), ptr(s), s.stride(0), ptr(t), t.stride(0), M, N, 1.0,
                 None, ptr(ds), N)
            ds = ds * drows.reshape(-1, 1)
        if ctx.needs_input_grad[1]:
            dt = torch.empty_like(t)
            call("rs_mse_rows", stream_handle(), ptr(t), t.stride(0), ptr(s), s.stride(0), M, N, 1.0,
                 None, ptr(dt), N)
            dt = dt * drows.reshape(-1, 1)
        return ds, dt


class KDLoss(nn.Module):
    """KDLoss()(student_predictions, teacher_predictions) (rough_rank/layer.py:272-279):
    per-sample mean squared error over the last axis -> [B]."""

    def forward(self, student_predictions, teacher_predictions):
        return _MSERowsFn.apply(student_predictions, teacher_predictions)


_BCE_WS: dict = {}

# Backward seeds known to hold exactly 1.0 for good (the Trainer's private loss.backward seed):
# the loss Functions return their pre-computed gradient as is for such a seed instead of
# launching a multiply by it.  The tensors are kept referenced, so their addresses never go to
# another tensor.
_UNIT_SEEDS: list = []
_UNIT_SEED_PTRS: set = set()


def register_unit_seed(t: torch.Tensor) -> None:
    """t: a 0-d float32 tensor holding 1.0 that nothing writes again."""
    if t.dim() != 0 or t.dtype != torch.float32:
        raise ValueError("a unit seed is a 0-d float32 tensor")
    _UNIT_SEEDS.append(t)
    _UNIT_SEED_PTRS.add(t.data_ptr())


def _times_seed(g: torch.Tensor, dl: torch.Tensor) -> torch.Tensor:
    if dl.dim() == 0 and dl.dtype == torch.float32 and dl.data_ptr() in _UNIT_SEED_PTRS:
        return g
    return g * dl


def _bce_workspace(device):
    """One persistent, zero-initialised workspace per device for rs_bce_clip_loss_ws (its size is
    bounded: 288 counter words + at most 64 block sums, so it is never reallocated under a
    captured graph that holds its address).  None while capturing before the first eager call
    (the single-workgroup rs_bce_clip_loss then runs)."""
    ws = _BCE_WS.get(device)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        n = int(_lib.load().rs_bce_clip_workspace_floats(1 << 40, 1))
        ws = torch.zeros(n, device=device, dtype=torch.float32)
        _BCE_WS[device] = ws
    return ws


class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, y, lo, hi, log_eps):
        p, y = _rows(p), _rows(y.float())
        M, T = p.shape
        loss = torch.empty(1, device=p.device)
        ds = torch.empty_like(p)
        ws = _bce_workspace(p.device)
        if ws is not None:
            call("rs_bce_clip_loss_ws", stream_handle(), ptr(p), ptr(y), M, T, lo, hi, log_eps, None,
                 None, ptr(loss), ptr(ds), ptr(ws), ws.numel())
        else:
            call("rs_bce_clip_loss", stream_handle(), ptr(p), ptr(y), M, T, lo, hi, log_eps, None,
                 None, ptr(loss), ptr(ds))
        ctx.save_for_backward(ds)
        return loss[0]

    @staticmethod
    def backward(ctx, dl):
        (ds,) = ctx.saved_tensors
        return _times_seed(ds, dl), None, None, None, None


def keras_bce(y_true, y_pred, eps=1e-7):
    """tf.keras.losses.BinaryCrossentropy() on probabilities (rough_rank/model.py:211-212):
    clip to [eps, 1 - eps], -(y log(p + eps) + (1 - y) log(1 - p + eps)), batch mean (T = 1)."""
    if y_pred.shape[-1] != 1:
        raise NotImplementedError("keras_bce is fused for one output column")
    return _BCEFn.apply(y_pred, y_true, eps, 1.0 - eps, eps)


def cross_entropy_sum(y_true, y_pred):
    """rank/multi_head/model.py:18-22 (and rank/ctr/base_model.py:7-12): -y log(p + 1e-6) -
    (1 - y) log(1 - p + 1e-6) summed over the last axis, mean over the batch; p unclipped."""
    return _BCEFn.apply(y_pred, y_true, -3.0e38, 3.0e38, 1e-6)


# ============================================================================================
# Fused multi-output loss total
# ============================================================================================
class LossTerm:
    """One output's share of a compiled Keras loss ``sum_k loss_weight_k * mean_batch(rows_k)``.
    ``launch(rows, grad, gscale)`` writes the output's per-row losses into ``rows`` [M] and the
    gradient of ``gscale * sum(rows)`` with respect to ``pred`` into ``grad`` (pred's shape,
    contiguous); every kernel used here (rs_bce_rows, rs_softmax_kl, rs_mse_rows) computes both in
    one launch."""

    __slots__ = ("pred", "weight", "launch")

    def __init__(self, pred, weight, launch):
        self.pred, self.weight, self.launch = pred, float(weight), launch


class _FusedLossFn(torch.autograd.Function):
    """Total of several LossTerms: one launch per term (rows + pre-scaled gradient), ONE
    rs_weighted_row_sum for the scalar; the backward scales every term's gradient by the incoming
    one in a single elementwise launch.  Replaces a reduction, a scale, an add and a backward
    multiply per output (staytime/model.py:85-89, rough_rank/model.py:210-214)."""

    @staticmethod
    def forward(ctx, terms, M, *preds):
        dev = preds[0].device
        K = len(terms)
        if not 1 <= K <= 6:
            raise ValueError("fused_loss takes 1 to 6 terms")
        R = torch.empty(K, M, device=dev)
        sizes = [p.numel() for p in preds]
        G = torch.empty(sum(sizes), device=dev)
        off = 0
        for k, (t, n) in enumerate(zip(terms, sizes)):
            t.launch(R[k], G[off:off + n], t.weight / M)
            off += n
        ws = [t.weight / M for t in terms] + [0.0] * (6 - K)
        out = torch.empty((), device=dev)
        call("rs_weighted_row_sum", stream_handle(), ptr(R), M, K, *ws, ptr(out))
        ctx.save_for_backward(G)
        ctx.sizes, ctx.shapes = sizes, [p.shape for p in preds]
        return out

    @staticmethod
    def backward(ctx, dl):
        (G,) = ctx.saved_tensors
        G = _times_seed(G, dl)
        grads, off = [], 0
        for n, shp in zip(ctx.sizes, ctx.shapes):
            grads.append(G[off:off + n].view(shp))
            off += n
        return (None, None, *grads)


def fused_loss(terms, M):
    """Scalar loss = sum_k terms[k].weight * mean_M(rows_k) (see LossTerm)."""
    return _FusedLossFn.apply(list(terms), int(M), *[t.pred for t in terms])


def bce_term(y_true, y_pred, weight=1.0, lo=-3.0e38, hi=3.0e38, log_eps=1e-6, sample_weight=None):
    """rs_bce_rows term: per row w_m sum_t [-y log(clip(p) + log_eps) - (1 - y) log(1 - clip(p) +
    log_eps)]; the defaults are staytime/model.py:33-36 cross_entropy, (eps, 1 - eps, eps) is
    tf.keras BinaryCrossentropy on probabilities (rough_rank/model.py:211-212)."""
    p = _rows(y_pred).contiguous()
    y = _rows(y_true.float()).contiguous()
    M, T = p.shape
    sw = sample_weight.reshape(-1).float().contiguous() if sample_weight is not None else None

    def launch(rows, grad, gscale):
        call("rs_bce_rows", stream_handle(), ptr(p), ptr(y), M, T, lo, hi, log_eps, ptr(sw), gscale,
             ptr(rows), ptr(grad))
    return LossTerm(p, weight, launch)


def keras_bce_term(y_true, y_pred, eps=1e-7, weight=1.0):
    return bce_term(y_true, y_pred, weight, eps, 1.0 - eps, eps)


def kd_mean_term(student, teacher, weight=1.0):
    """mean over the batch of KDLoss rows (rough_rank/layer.py:272-279, model.py:214: the
    'distill' output's y_pred_loss) with the teacher stop-gradient (model.py:166)."""
    s = _rows(student)
    t = _rows(teacher.detach())
    M, N = s.shape

    def launch(rows, grad, gscale):
        call("rs_mse_rows", stream_handle(), ptr(s), s.stride(0), ptr(t), t.stride(0), M, N, gscale,
             ptr(rows), ptr(grad), N)
    return LossTerm(s, weight, launch)
