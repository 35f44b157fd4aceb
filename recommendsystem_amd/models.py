"""Ranking-model builders of the reference, re-composed from the MI355X ops.

    MultiHeadRanker   rank/multi_head/multidnn.py:14-259 (AUTOINT / create_autoint_sub_model)
    DSSM              rough_rank/model.py:16-198 (user/item PLE towers, CrossNet teacher,
                      shallow student, KD)
    StaytimeMTL       staytime/VideoDnn.py:27-302 (mtl_net / create_moe_sub_model)

Each model is an nn.Module whose ``forward(batch)`` returns the reference's named outputs and
whose ``loss(batch)`` returns the compiled Keras loss (losses x loss_weights, sample weights,
kernel regularisers handled by the trainer through rs_l1l2_grad).  Every compute op runs in
librecsys_amd.so; torch only allocates, slices and concatenates activations.

Layers that read the same input with the same activation are fused into one GEMM
(``SharedInputDense``: the Keras kernels are column blocks of one [K, sum N] matrix), e.g. the
three staytime experts' first layers plus the three MMoE gate nets' first layers are one
[1712, 960] GEMM, and the six ppnet first-gate layers one [224, 1152] GEMM.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Sequence

import torch
from torch import nn

from ._lib import call, ptr, stream_handle
from .din import StaytimeDIN
from .embedding import EmbeddingFeatures, SequenceEmbedding, SparseAdaGrad, SparseAdam, SparseTable
from .layers import (Dense, GradSink, InteractingLayer, _act_code, _DenseFn, _row_major, gather_multi,
                     grouped_dense)
from .params import FlatBlock, glorot_uniform_, grads_contiguous
from . import _lib
from .towers import (DNN, PLE, CrossNet, DeepCrossLayer, ExpertGateLayer, FFMBlock, KDLoss,
                     SENetFM, StaytimeHead, _rows, _split_grads, bce_term, cross_entropy_sum, fused_loss,
                     gated, gated_group, kd_mean_term, keras_bce, keras_bce_term)


# ============================================================================================
# small fused pieces
# ============================================================================================
class _SplitColsFn(torch.autograd.Function):
    """Column blocks of y [B, sum sizes] (views); the backward is ONE concat of the
    blocks' gradients (autograd's per-view backward would zero-fill a full-width gradient per block
    and add them up: 2N elementwise launches per step instead of one)."""

    @staticmethod
    def forward(ctx, y, sizes):
        ctx.sizes = sizes
        return tuple(torch.split(y, sizes, dim=1))

    @staticmethod
    def backward(ctx, *grads):
        B = next(g.shape[0] for g in grads if g is not None)
        ref = next(g for g in grads if g is not None)
        parts = [g if g is not None else ref.new_zeros(B, n) for g, n in zip(grads, ctx.sizes)]
        return torch.cat(parts, dim=1), None


class _StaytimeFrontFn(torch.autograd.Function):
    """The staytime trunk's reads of the field embeddings emb [B, F, 32] in one Function
    (VideoDnn.py:11-25, 45-47, 57-77, 99-105, 127): general = emb[:, :, 0:16] and the DIN queries
    general[:, q] (views), the gate input emb[:, bias, 16:32] (one column gather) and the fused
    FFM + user x item multiply over the user / item fields.  Backward: ONE gather-sum kernel
    writes every element of d_emb from the general, gate and query gradients, then the FFM
    backward adds its share in place -- instead of a zero fill, a copy, an add + copy per query, an
    index_add, the FFM's own zero-filled d_emb and autograd's add of the two."""

    @staticmethod
    def forward(ctx, emb, Wx, bx, Wy, by, front):
        B, F, W = emb.shape
        emb = emb.contiguous()
        x2 = emb.view(B, F * W)
        ffm = front["ffm"]
        gate = torch.empty(B, front["gate_cols"].numel(), device=emb.device)
        call("rs_gather_columns", stream_handle(), ptr(x2), F * W, B, ptr(front["gate_cols"]),
             gate.shape[1], ptr(gate), gate.shape[1])
        P = ffm.NU * ffm.NI
        y = torch.empty(B, P * ffm.dim, device=emb.device)
        mu = torch.empty(B, ffm.NU * 16, device=emb.device)
        call("rs_ffm_fwd", stream_handle(), ptr(x2), F * W, B, ffm.NU, ffm.NI, 16, ffm.dim,
             ptr(ffm.cols), ptr(Wx), ptr(bx), ptr(Wy), ptr(by), ptr(y), P * ffm.dim, ptr(mu),
             ffm.NU * 16)
        ctx.save_for_backward(emb, Wx, bx, Wy, by)
        ctx.front = front
        general = emb[:, :, 0:16]
        return (general, gate, *[emb[:, q, 0:16] for q in front["qidx"]], y, mu)

    @staticmethod
    def backward(ctx, dgen, dgate, *rest):
        emb, Wx, bx, Wy, by = ctx.saved_tensors
        front = ctx.front
        nq = len(front["qidx"])
        dqs, dy, dmu = rest[:nq], rest[nq], rest[nq + 1]
        B, F, W = emb.shape
        dev = emb.device
        srcs = []
        for g, width in [(dgen, F * 16), (dgate, front["gate_cols"].numel())] + [(d, 16) for d in dqs]:
            if g is None:
                g = torch.zeros(B, width, device=dev)
            g = g.reshape(B, width) if g.is_contiguous() else g.contiguous().reshape(B, width)
            srcs.append(g)
        d_emb = torch.empty(B, F, W, device=dev)
        ptrs = (ctypes.c_void_p * len(srcs))(*[g.data_ptr() for g in srcs])
        lds = (ctypes.c_int64 * len(srcs))(*[g.stride(0) for g in srcs])
        call("rs_gather_sum_columns", stream_handle(), len(srcs), ctypes.addressof(ptrs),
             ctypes.addressof(lds), ptr(front["fanout_map"]), B, F * W, ptr(d_emb), F * W)
        ffm = front["ffm"]
        params = (Wx, bx, Wy, by)
        if dy is None and dmu is None:
            return (d_emb, None, None, None, None, None)
        P = ffm.NU * ffm.NI
        dy = _row_major(dy) if dy is not None else torch.zeros(B, P * ffm.dim, device=dev)
        dmu = _row_major(dmu) if dmu is not None else None
        lib = _lib.load()
        ws_n = int(lib.rs_ffm_bwd_workspace_floats(B, ffm.NU, ffm.NI, 16, ffm.dim))
        ws = torch.empty(max(ws_n, 1), device=dev)
        block = grads_contiguous(params)
        dpar = block if block is not None else torch.empty(sum(p.numel() for p in params), device=dev)
        call("rs_ffm_bwd", stream_handle(), ptr(emb), F * W, B, ffm.NU, ffm.NI, 16, ffm.dim,
             ptr(ffm.cols), ptr(Wx), ptr(bx), ptr(Wy), ptr(by), ptr(dy), dy.stride(0), ptr(dmu),
             dmu.stride(0) if dmu is not None else ffm.NU * 16, ptr(d_emb), F * W, 1, ptr(dpar),
             1 if block is not None else 0, ptr(ws), ws_n)
        g = (None,) * 4 if block is not None else tuple(_split_grads(params, dpar))
        return (d_emb, *g, None)


def split_cols(y, sizes):
    return list(_SplitColsFn.apply(y, list(sizes)))


class SharedInputDense(nn.Module):
    """Several Keras Dense(u_i, act) layers applied to the SAME input: one [K, sum u] kernel,
    one GEMM; ``forward`` returns the per-layer column views."""

    def __init__(self, units: Sequence[int], activation=None, seed=0, device=None,
                 init="glorot_uniform"):
        super().__init__()
        self.units = [int(u) for u in units]
        self.act = _act_code(activation)
        self.seed, self._device, self.init = seed, device, init
        self.built = False

    def build(self, input_shape, device=None):
        K, N = int(input_shape[-1]), sum(self.units)
        device = device or self._device or torch.device("cuda")
        blk = FlatBlock([(K, N), (N,)], device)
        self.kernel, self.bias = blk.params()
        gen = torch.Generator().manual_seed(self.seed)
        off = 0
        for u in self.units:
            t = torch.empty(K, u)
            glorot_uniform_(t, K, u, gen)
            with torch.no_grad():
                self.kernel[:, off:off + u].copy_(t)
            off += u
        self.input_dim = K
        self.built = True

    def layer_kernel(self, i):
        o = sum(self.units[:i])
        return self.kernel[:, o:o + self.units[i]]

    def layer_bias(self, i):
        o = sum(self.units[:i])
        return self.bias[o:o + self.units[i]]

    def forward(self, x):
        if not self.built:
            self.build(tuple(x.shape), device=x.device)
        y = _DenseFn.apply(_rows(x), self.kernel, self.bias, self.act)
        return split_cols(y, self.units)


class _GroupedHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, T, D, act):
        x = _rows(x)
        M = x.shape[0]
        y = torch.empty(M, T, device=x.device)
        call("rs_grouped_head_fwd", stream_handle(), ptr(x), x.stride(0), M, T, D, ptr(W), ptr(b), act,
             ptr(y), T)
        ctx.save_for_backward(x, W, b, y)
        ctx.cfg = (T, D, act)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, b, y = ctx.saved_tensors
        T, D, act = ctx.cfg
        M = x.shape[0]
        dy = dy.contiguous()
        dx = torch.empty(M, T * D, device=x.device)
        ws_n = int(_lib.load().rs_grouped_head_bwd_workspace_floats(M, T, D))
        ws = torch.empty(max(ws_n, 1), device=x.device)
        block = grads_contiguous((W, b))
        dp = block if block is not None else torch.empty(T * D + T, device=x.device)
        call("rs_grouped_head_bwd", stream_handle(), ptr(x), x.stride(0), M, T, D, ptr(W), ptr(y), T, act,
             ptr(dy), T, ptr(dx), T * D, ptr(dp), 1 if block is not None else 0, ptr(ws), ws_n)
        if block is not None:
            return dx, None, None, None, None, None
        return dx, dp[:T * D].view(W.shape), dp[T * D:].view(b.shape), None, None, None


class GroupedHeads(nn.Module):
    """T Keras Dense(1, act) towers, tower t on columns [t*D, t*D + D) of its input
    (rank/multi_head/multidnn.py:122-204).  W [T, D] (row t = tower t's [D, 1] kernel), b [T]."""

    def __init__(self, T, D, activation="sigmoid", seed=0, device=None):
        super().__init__()
        self.T, self.D = int(T), int(D)
        self.act = _act_code(activation)
        device = device or torch.device("cuda")
        blk = FlatBlock([(self.T, self.D), (self.T,)], device)
        self.W, self.b = blk.params()
        gen = torch.Generator().manual_seed(seed)
        for t in range(self.T):
            k = torch.empty(self.D, 1)
            glorot_uniform_(k, self.D, 1, gen)
            with torch.no_grad():
                self.W[t].copy_(k[:, 0])

    def forward(self, x):
        return _GroupedHeadFn.apply(x, self.W, self.b, self.T, self.D, self.act)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        x = x.contiguous().float()
        y = torch.empty_like(x)
        call("rs_act_fwd", stream_handle(), ptr(x), x.numel(), act, ptr(y))
        ctx.save_for_backward(y)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        call("rs_act_bwd", stream_handle(), ptr(y), ptr(dy.contiguous()), y.numel(), ctx.act, ptr(dx))
        return dx, None


def sigmoid(x):
    return _ActFn.apply(x, 2)


class _RowSelectFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mask, a, b):
        a, b = _rows(a), _rows(b)
        mask = mask.reshape(-1).float().contiguous()
        M, N = a.shape
        y = torch.empty(M, N, device=a.device)
        call("rs_row_select", stream_handle(), ptr(mask), ptr(a), a.stride(0), ptr(b), b.stride(0), M, N,
             ptr(y), N, None, None, None)
        ctx.save_for_backward(mask)
        ctx.shape = (M, N)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        M, N = ctx.shape
        da = torch.empty(M, N, device=dy.device)
        db = torch.empty(M, N, device=dy.device)
        call("rs_row_select", stream_handle(), ptr(mask), None, 0, None, 0, M, N, None, N,
             ptr(dy.contiguous()), ptr(da), ptr(db))
        return None, da, db


def row_select(mask, a, b):
    """tf.where(mask == 1, a, b) per row (rough_rank/model.py:52-53)."""
    return _RowSelectFn.apply(mask, a, b)


# ============================================================================================
# H5: rank/multi_head AUTOINT
# ============================================================================================
@dataclass
class MultiHeadConfig:
    num_fields: int = 200            # config 3
    embed_dim: int = 8               # embedding_columns_builder(..., 8, combiner='mean') :227
    vocab_per_field: int = 265_000   # rank/ctr/base_model.py:206 bucket size
    dnn_hidden_units: Sequence[int] = (32, 16)   # AUTOINT default :214
    expert_num: int = 7              # :79 (expert_num + 1 Dense layers built, 7 stacked :89)
    expert_units: int = 32
    num_label: int = 7               # :97
    dropout_rate: float = 0.2        # :54
    lr_dense: float = 1e-5           # rank/multi_head/model.py:52
    lr_sparse: float = 5e-5          # :235


class MultiHeadRanker(nn.Module):
    """create_autoint_sub_model + AUTOINT (rank/multi_head/multidnn.py:14-259).

    emb [B, F, 8] (mean of a VarLen id list per field) -> IL(1, 8, 2, dropout .2, res) ->
    flatten; deep Flatten -> Dense(32) -> Dense(16) relu with L1L2(1e-5, 1e-5); result =
    concat [deep, autoint] (16 + 8F); 7 experts Dense(32, relu) + 7 gates Dense(7, softmax)
    (TruncatedNormal(0.001), L2(0.01)) -> one GEMM + rs_gate_mix; 7 towers Dense(1, sigmoid).
    The 8th expert Dense of :81 is built by Keras but not connected to any output, so it is not
    part of the trained model and is not materialised here."""

    def __init__(self, cfg: MultiHeadConfig | None = None, device=None, seed=0, max_touched=None):
        super().__init__()
        self.cfg = cfg = cfg or MultiHeadConfig()
        dev = torch.device(device or "cuda")
        F, E = cfg.num_fields, cfg.embed_dim
        self.table = SparseTable(F * cfg.vocab_per_field, E, SparseAdam(cfg.lr_sparse), device=dev,
                                 seed=seed, max_touched=max_touched)
        # list mode: the scan form (a 212 MB flag sweep of the 53 M-row table instead of claims +
        # the touched list) measured 1.72 vs 1.656 ms per step (profiles/r06/push/mh_scan.txt);
        # RS_MH_SCAN=1 selects it at world 1 (A/B)
        self.table.prefer_scan = os.environ.get("RS_MH_SCAN", "0") == "1"
        self.embedding = EmbeddingFeatures(self.table, [cfg.vocab_per_field] * F, combiner="mean")
        self.interact = InteractingLayer(1, E, 2, use_dropout=True, dropout_rate=cfg.dropout_rate,
                                         use_res=True, seed=seed + 1, device=dev)
        self.interact.build((1, F, E), device=dev)
        self.deep = nn.ModuleList()
        d_in = F * E
        for i, u in enumerate(cfg.dnn_hidden_units):
            layer = Dense(u, "relu", seed=seed + 10 + i, device=dev, name=f"dnn_{i}")
            layer.build((1, d_in), device=dev)
            self.deep.append(layer)
            d_in = u
        K = d_in + F * E
        self.mix = ExpertGateLayer(cfg.expert_num, cfg.expert_units,
                                   [list(range(cfg.expert_num))] * cfg.num_label, "relu",
                                   expert_init=("truncated_normal", 0.001),
                                   gate_init=("truncated_normal", 0.001), seed=seed + 30, device=dev)
        self.mix.build((1, K), device=dev)
        self.towers = GroupedHeads(cfg.num_label, cfg.expert_units, "sigmoid", seed=seed + 40, device=dev)
        self.result_dim = K

    def tables(self):
        return [self.table]

    def regularizers(self):
        """(param, l1, l2): L1L2(1e-5, 1e-5) on the deep kernels (:62-63), L2(0.01) on the
        expert and gate kernels (:85,103)."""
        return [(l.kernel, 1e-5, 1e-5) for l in self.deep] + [(self.mix.kernel, 0.0, 0.01)]

    def forward(self, ids, offsets):
        x0 = self.embedding(ids, offsets)                       # [B, F, 8]
        B = x0.shape[0]
        # :60-63 the deep tower; its first Dense also adds the interacting layers' dx0 in its
        # backward (GradSink: no separate sum of the two [B, F E] gradients)
        sink = GradSink() if self.deep else None
        deep = x0.reshape(B, -1)
        for k, layer in enumerate(self.deep):
            deep = layer(deep, grad_sink=sink) if k == 0 else layer(deep)
        # :54-56 interacting layers, :71 concat [deep, autoint]: the layer writes its output
        # into the concat directly
        result = self.interact.forward_concat(deep, x0, grad_sink=sink)
        gated_out = self.mix.forward_flat(result)               # :77-120, the 7 outputs side by side
        return self.towers(gated_out)                           # :122-204 -> [B, 7]

    def loss(self, ids, offsets, labels):
        """rank/multi_head/model.py:18-22 per output, summed by Keras over the 7 outputs."""
        return cross_entropy_sum(labels, self.forward(ids, offsets))


# ============================================================================================
# H8: rough_rank DSSM (two-tower pre-ranker with distillation)
# ============================================================================================
@dataclass
class DSSMConfig:
    user_fields: int = 33            # user [B, 33*16 = 528]
    item_fields: int = 19            # item [B, 19*16 = 304]
    emb_dim: int = 16                # C.USER_OUTPUT_DIM / ITEM_OUTPUT_DIM
    output_dim: int = 16
    lr_dense: float = 1e-4           # rough_rank/model.py:209
    lr_sparse: float = 1e-3          # :106


class UserItemTower(nn.Module):
    """create_tower (rough_rank/model.py:37-67): PLE(num_tasks, 4 shared, 4 specific, (32,))
    then DNN((output_dim,), output_activation='linear') per task; with a mask input the two task
    embeddings are selected per row by tf.where(mask == 1, task1, task0)."""

    def __init__(self, in_dim, num_tasks, output_dim=16, seed=0, device=None):
        super().__init__()
        self.ple = PLE(num_tasks=num_tasks, num_shared_experts=4, num_specific_experts=4,
                       expert_dnn_units=(32,), gate_dnn_units=(), expert_dnn_params=dict(),
                       gate_dnn_params=dict(), seed=seed, device=device)
        self.ple.mix.build((1, in_dim), device=device)
        self.heads = nn.ModuleList()
        for t in range(num_tasks):
            d = DNN((output_dim,), output_activation="linear", l2_reg=0, dropout_rate=0, seed=seed + 7 + t,
                    device=device)
            d.build((1, 32), device=device)
            self.heads.append(d)

    def forward(self, x, mask=None):
        outs = self.ple(x)
        embs = [h(o) for h, o in zip(self.heads, outs)]
        if mask is not None:
            return row_select(mask, embs[1], embs[0])
        return embs[0]


class DSSM(nn.Module):
    """DSSM() (rough_rank/model.py:118-198) on a [B, user_fields + item_fields, 16] embedding
    input whose field order is the teacher's sorted order; ``user_idx`` / ``item_idx`` pick each
    tower's fields (dict_to_sorted_list of the tower's own inputs)."""

    def __init__(self, cfg: DSSMConfig | None = None, user_idx=None, item_idx=None, device=None, seed=0):
        super().__init__()
        self.cfg = cfg = cfg or DSSMConfig()
        dev = torch.device(device or "cuda")
        nu, ni, E = cfg.user_fields, cfg.item_fields, cfg.emb_dim
        self.user_idx = torch.tensor(user_idx if user_idx is not None else list(range(nu)), device=dev)
        self.item_idx = torch.tensor(item_idx if item_idx is not None else list(range(nu, nu + ni)), device=dev)
        self._plan_key, self._plan = None, None
        self.user = UserItemTower(nu * E, 2, cfg.output_dim, seed=seed, device=dev)
        self.item = UserItemTower(ni * E, 1, cfg.output_dim, seed=seed + 100, device=dev)
        D = (nu + ni) * E
        self.cross = CrossNet(layer_num=2, device=dev)                          # :24
        self.cross.build((1, D), device=dev)
        self.t1 = Dense(128, "relu", seed=seed + 201, device=dev)
        self.t2 = Dense(64, "relu", seed=seed + 202, device=dev)
        self.t3 = Dense(16, None, seed=seed + 203, device=dev)
        self.t4 = Dense(1, None, seed=seed + 204, device=dev, name="pred_teacher")
        self.s1 = Dense(32, "relu", seed=seed + 301, device=dev, name="shallow_dnn_0")
        self.s2 = Dense(1, None, seed=seed + 302, device=dev, name="logit_shallow")
        for layer, k in ((self.t1, D), (self.t2, 128), (self.t3, 64 + D), (self.t4, 16),
                         (self.s1, 2 * cfg.output_dim), (self.s2, 32)):
            layer.build((1, k), device=dev)
        self.kd = KDLoss()

    def regularizers(self):
        return []

    def _plans(self, nf, width):
        """Column plans over a [B, nf * width] lookup output whose first 16 columns per field are
        this model's embedding: user fields, item fields, and all fields (the teacher's input)."""
        key = (nf, width)
        if self._plan_key != key:
            dev = self.user_idx.device
            d = self.cfg.emb_dim

            def cols(fields):
                return torch.tensor([int(f) * width + c for f in fields for c in range(d)],
                                    dtype=torch.int32, device=dev)
            self._plan = (cols(self.user_idx.tolist()), cols(self.item_idx.tolist()),
                          cols(range(nf)))
            self._plan_key = key
        return self._plan

    def forward(self, emb, mask, with_kd=True):
        """emb [B, nu + ni, 16] (or any [B, F, >= 16] whose columns 0:16 per field are the
        embedding -- the joint model's [B, 52, 32] lookup); mask [B, 1] (dense feature 4575).
        Returns the reference's outputs {'student', 'teacher', 'distill'} plus the logits."""
        B, nf, width = emb.shape
        emb = emb.contiguous()
        # index_select + reshape of the user / item fields and the teacher's flatten (:21-22,
        # :145-149) as column gathers of the lookup rows: one launch each, one fused backward
        ux, ix, wc = gather_multi(emb.reshape(B, nf * width), self._plans(nf, width))
        heads = [h.layers for h in list(self.user.heads) + list(self.item.heads)]
        if all(len(h) == 1 for h in heads):
            # the towers' per-task output DNNs (one Dense each) as one grouped launch per pass
            uo, io = self.user.ple(ux), self.item.ple(ix)
            he = grouped_dense([h[0] for h in heads], list(uo) + list(io))
            nu_t = len(self.user.heads)
            user_emb = row_select(mask, he[1], he[0]) if mask is not None else he[0]  # :145-146
            item_emb = he[nu_t]                                                  # :148-149
        else:
            user_emb = self.user(ux, mask)
            item_emb = self.item(ix)
        cross = self.cross(wc)                                                   # :24
        deep = self.t2(self.t1(wc))                                              # :25-26
        # the teacher's and the student's last two layers pairwise grouped (independent chains)
        t3o, s1o = grouped_dense([self.t3, self.s1], [torch.cat([deep, cross], dim=1),   # :27-29
                                                      torch.cat([user_emb, item_emb], dim=1)])  # :73-81
        t_logit, s_logit = grouped_dense([self.t4, self.s2], [t3o, s1o])
        distill = self.kd(s_logit, t_logit.detach()) if with_kd else None        # :175-176
        return {"student": sigmoid(s_logit), "teacher": sigmoid(t_logit), "distill": distill,
                "student_logit": s_logit, "teacher_logit": t_logit}

    def loss_terms(self, emb, mask, labels):
        """create_model losses (rough_rank/model.py:210-214) as fused LossTerms: BCE(student) +
        BCE(teacher) + y_pred_loss(distill) = mean of the per-sample KD loss."""
        out = self.forward(emb, mask, with_kd=False)
        return [keras_bce_term(labels, out["student"]), keras_bce_term(labels, out["teacher"]),
                kd_mean_term(out["student_logit"], out["teacher_logit"])]

    def loss(self, emb, mask, labels):
        return fused_loss(self.loss_terms(emb, mask, labels), emb.shape[0])


# ============================================================================================
# H9: staytime mtl_net
# ============================================================================================
STAYTIME_BINS = [-19.0 + 0.5 * i for i in range(400)]   # staytime/config.py:18-42 (-19 .. 180.5)


@dataclass
class StaytimeConfig:
    num_fields: int = 91             # len(C.SLOTS)
    emb_dim: int = 32                # fetch_embeddings_seq dimension=32 (:229-230)
    seq_len: int = 50                # mtl_net(..., 50, ...) staytime/model.py:71
    num_seq: int = 3                 # C.SEQ_SLOTS
    user_fields: Sequence[int] = (0, 14, 37, 1)       # USER_SLOTS positions in sorted SLOTS
    item_fields: Sequence[int] = (15, 17, 29, 24)     # ITEM_SLOTS positions
    bias_fields: Sequence[int] = (64, 1, 37, 62, 0, 67, 65, 66, 63, 29, 17, 15, 14, 24)
    query_fields: Sequence[int] = (15, 17, 29)        # '1591', '1593', '1737' (:53-55)
    hidden_units: Sequence[int] = (256, 128)          # create_model_func dnn_hidden_units
    num_experts: int = 3
    num_tasks: int = 3
    loss_weights: Sequence[float] = (2.0, 2.0, 1.0)   # staytime/model.py:85-87
    lr_dense: float = 5e-4                            # staytime/model.py:72


class StaytimeMTL(nn.Module):
    """create_moe_sub_model (staytime/VideoDnn.py:27-215) over field embeddings emb
    [B, 91, 32] (mean-pooled) and three DIN sequences [B, 50, 32] with masks [B, 50].

    general_f = emb[:, f, 0:16]; bias = emb[:, bias_fields, 16:32] (224 wide); three DIN pools
    (queries = general of '1591' / '1593' / '1737'); SENet reweight + FM; user x item multiply;
    FFM (16 pairs x 8); concat -> 1712; 3 ppnet-gated experts [256, 128]; 3 MMoE gates
    [64, 32] -> softmax(3); DCN(3); staytime head (400 bins) on [mmoe_0, cross]; shortplay /
    longplay sigmoid heads on [fm_logit, Dense(1, relu)(mmoe_t)]."""

    def __init__(self, cfg: StaytimeConfig | None = None, device=None, seed=0):
        super().__init__()
        self.cfg = cfg = cfg or StaytimeConfig()
        dev = torch.device(device or "cuda")
        F = cfg.num_fields
        self.dins = nn.ModuleList()
        for s in range(cfg.num_seq):
            d = StaytimeDIN(seed=seed + s, device=dev)
            d.build((1, cfg.seq_len, 16), device=dev)
            self.dins.append(d)
        self.senet = SENetFM(F, seed=seed + 10, device=dev)
        self.senet.squeeze.build((1, F * 16), device=dev)
        self.senet.excite.build((1, int(F / 4)), device=dev)
        self.ffm = FFMBlock(list(cfg.user_fields), list(cfg.item_fields), 8, True, seed=seed + 20,
                            device=dev, field_stride=cfg.emb_dim)
        self.concat_dim = D = F * 16 + 16 + 4 * 16 + 16 * 8 + cfg.num_seq * 16     # 1712
        self.gate_dim = G = len(cfg.bias_fields) * 16                              # 224
        H = list(cfg.hidden_units)
        NE = cfg.num_experts
        # first layers sharing concated_input: 3 experts' layer 0 + 3 MMoE gates' layer 0 (64)
        self.first = SharedInputDense([H[0]] * NE + [64] * cfg.num_tasks, "relu", seed=seed + 30, device=dev)
        self.first.build((1, D), device=dev)
        # ppnet first-gate layers, all on gate_input: expert i, layer j
        self.pp1 = SharedInputDense([u for _ in range(NE) for u in H], "relu", seed=seed + 40, device=dev)
        self.pp1.build((1, G), device=dev)
        self.pp2 = nn.ModuleList()
        self.exp_rest = nn.ModuleList()
        for i in range(NE):
            for j, u in enumerate(H):
                g2 = Dense(u, "sigmoid", seed=seed + 50 + 10 * i + j, device=dev)
                g2.build((1, u), device=dev)
                self.pp2.append(g2)
                if j > 0:
                    e = Dense(u, "relu", seed=seed + 80 + 10 * i + j, device=dev)
                    e.build((1, H[j - 1]), device=dev)
                    self.exp_rest.append(e)
        self.gate_l2 = nn.ModuleList()
        self.gate_out = nn.ModuleList()
        for t in range(cfg.num_tasks):
            g = Dense(32, "relu", seed=seed + 110 + t, device=dev)
            g.build((1, 64), device=dev)
            o = Dense(NE, None, seed=seed + 120 + t, device=dev)  # softmax applied by rs_gate_mix
            o.build((1, 32), device=dev)
            self.gate_l2.append(g)
            self.gate_out.append(o)
        self.sel = torch.arange(NE, dtype=torch.int32, device=dev).repeat(cfg.num_tasks)
        self.dcn = DeepCrossLayer(num_layer=3, seed=seed + 130, device=dev)
        self.dcn.build((1, D), device=dev)
        self.head = StaytimeHead(STAYTIME_BINS, seed=seed + 140, device=dev)
        self.head.dense.build((1, H[-1] + D), device=dev)
        self.deep_logit = nn.ModuleList()
        self.task_out = nn.ModuleList()
        for t in (1, 2):
            dl = Dense(1, "relu", seed=seed + 150 + t, device=dev)
            dl.build((1, H[-1]), device=dev)
            to = Dense(1, "sigmoid", seed=seed + 160 + t, device=dev)
            to.build((1, 2), device=dev)
            self.deep_logit.append(dl)
            self.task_out.append(to)
        dev_ = dev
        self.bias_idx = torch.tensor(list(cfg.bias_fields), device=dev_)
        self.query_idx = list(cfg.query_fields)

    def regularizers(self):
        return []

    def _front(self, F, W):
        """Device plans of _StaytimeFrontFn for emb [B, F, W]: the gate gather columns and the
        fan-out map [2 + len(query_fields), F * W] (general, gate, queries -> emb columns)."""
        key = (F, W)
        if getattr(self, "_front_key", None) != key:
            dev = self.bias_idx.device
            bias = [int(f) for f in self.cfg.bias_fields]
            gate_cols = [f * W + 16 + c for f in bias for c in range(16)]
            nsrc = 2 + len(self.query_idx)
            mp = [[-1] * (F * W) for _ in range(nsrc)]
            for f in range(F):
                for c in range(16):
                    mp[0][f * W + c] = f * 16 + c
            for slot, f in enumerate(bias):
                if mp[1][f * W + 16] != -1:
                    raise ValueError("bias fields must be distinct")
                for c in range(16):
                    mp[1][f * W + 16 + c] = slot * 16 + c
            for k, q in enumerate(self.query_idx):
                for c in range(16):
                    mp[2 + k][int(q) * W + c] = c
            self._front_plan = {
                "gate_cols": torch.tensor(gate_cols, dtype=torch.int32, device=dev),
                "fanout_map": torch.tensor(mp, dtype=torch.int32, device=dev),
                "qidx": [int(q) for q in self.query_idx], "ffm": self.ffm}
            self._front_key = key
        return self._front_plan

    def _trunk(self, emb, seqs, masks):
        cfg = self.cfg
        B, F, _ = emb.shape
        # general = emb[:, :, 0:16] (:47); gate input = bias fields' [16:32] (:45-46,127); DIN
        # queries = general of the query fields (:57-77)
        nq = len(self.query_idx)
        general, gate_input, *rest = _StaytimeFrontFn.apply(emb, self.ffm.Wx, self.ffm.bx,
                                                            self.ffm.Wy, self.ffm.by,
                                                            self._front(F, emb.shape[2]))
        queries, (ffm, mult) = rest[:nq], rest[nq:]
        # the DIN reads columns 0:16 of the 32-wide sequence rows in place and its backward writes
        # the full-width gradient (no autograd slice: zero fill + strided copy per sequence)
        din = [self.dins[s](queries[s], seqs[s], masks[s], wide=True)
               for s in range(len(self.query_idx))]
        rew, cross_term, fm_logit = self.senet(general)                            # :81-115
        concated = torch.cat([rew, cross_term, mult, ffm] + din, dim=1)            # :122-123
        H, NE, L = list(cfg.hidden_units), cfg.num_experts, len(cfg.hidden_units)
        firsts = self.first(concated)
        pp1 = self.pp1(gate_input)
        # the per-expert / per-task layers as grouped launches (one per pass for each group):
        # expert i, layer j: gate = pp2[i L + j](pp1[i L + j]) (:134-138); deep = exp_rest[i (L-1)
        # + j - 1](deep) for j > 0; deep = gated(deep, gate, 2) (:139-146)
        gs = grouped_dense(self.pp2, [pp1[q] for q in range(NE * L)])
        deeps = [firsts[i] for i in range(NE)]
        for j in range(L):
            if j > 0:
                deeps = grouped_dense([self.exp_rest[i * (L - 1) + j - 1] for i in range(NE)], deeps)
            deeps = gated_group(deeps, [gs[i * L + j] for i in range(NE)], 2.0)
        T = cfg.num_tasks
        gates = grouped_dense(self.gate_out,
                              grouped_dense(self.gate_l2, [firsts[NE + t] for t in range(T)]))
        return concated, fm_logit, deeps, gates

    def forward(self, emb, seqs, masks, with_loss=False, labels=None):
        """Named outputs, or with ``with_loss`` (loss, outputs)."""
        if with_loss:
            terms, outs = self._outputs(emb, seqs, masks, True, labels)
            return fused_loss(terms, emb.shape[0]), outs   # fills outs["staytime"] (P)
        return self._outputs(emb, seqs, masks)

    def _outputs(self, emb, seqs, masks, with_loss=False, labels=None):
        cfg = self.cfg
        concated, fm_logit, experts, gates = self._trunk(emb, seqs, masks)
        from .towers import _MixFn
        Z = torch.cat(experts + gates, dim=1)           # [experts (:150) | gate logits]: one copy
        mm = _MixFn.apply(Z, self.sel, cfg.num_experts, cfg.hidden_units[-1], cfg.num_tasks,
                          cfg.num_experts, 0)                                       # :153-164
        Hh = cfg.hidden_units[-1]
        mmoe = split_cols(mm, [Hh] * cfg.num_tasks)
        # :167-168 cross = DeepCrossLayer(concated); ext = concat([mmoe[0], cross]): the cross
        # kernel writes into ext directly
        ext = self.dcn.forward_concat(mmoe[0], concated)
        dl = grouped_dense(self.deep_logit, [mmoe[1], mmoe[2]])
        short, long_ = grouped_dense(self.task_out, [torch.cat([fm_logit, dl[0]], dim=1),  # :182-185
                                                     torch.cat([fm_logit, dl[1]], dim=1)])  # :188-191
        if not with_loss:
            return {"staytime": self.head(ext), "shortplay": short, "longplay": long_}
        y_stay, y_short, y_long, sw = labels
        w = cfg.loss_weights
        # custom_kl_loss + 2 x cross_entropy with loss_weights and sample weights (model.py:20-36,
        # 85-89) as fused LossTerms: one launch per output + one for the weighted total
        kl, P = self.head.loss_term(ext, y_stay, sw, loss_weight=w[0])
        terms = [kl, bce_term(y_short, short, w[1], sample_weight=sw),
                 bce_term(y_long, long_, w[2], sample_weight=sw)]
        return terms, {"staytime": P, "shortplay": short, "longplay": long_}

    def loss_terms(self, emb, seqs, masks, y_stay, y_short, y_long, sample_weight=None):
        return self._outputs(emb, seqs, masks, True, (y_stay, y_short, y_long, sample_weight))[0]

    def loss(self, emb, seqs, masks, y_stay, y_short, y_long, sample_weight=None):
        return self.forward(emb, seqs, masks, True, (y_stay, y_short, y_long, sample_weight))[0]
