"""The rank/ctr production model and rank/finish DeepFM, composed
from librecsys_amd.so kernels (csrc/front_end.hip plus the shared Dense / InteractingLayer /
gating / mixture kernels).

    RankCtrFrontEnd   rank/ctr BaseModel.__init__ (base_model.py:29-159): per-feature VarLen
                      lookups into slot tables (featureid_to_slot sharing, base_model.py:89-102)
                      of width max_embed_size, then the column plans of the structure fields,
                      the gate fields and the bias groups (rs_gather_columns).
    RankCtrModel      rank/ctr Model.model_layer (model_init.py:19-162): SENet over the
                      structure fields, per-field Dense(8) -> InteractingLayer(1, 8, 2), ppnet
                      gates, the gated deep tower, user x item multiply, CAN per-sample
                      matmuls, 3-expert ppnet-gated MMoE, two gated task towers, clipped
                      sigmoid outputs and the summed cross_entropy losses.
    FMLayer           rank/finish FMLayer(Dense) (videodnn.py:23-52): learned fm_matrix [D, 8],
                      0.5 * sum((xV)^2 - x^2 V^2) + Dense(1) linear term.
    DeepFM            rank/finish create_deepFM_sub_model / DEEPFM (videodnn.py:69-196).

torch only allocates, slices and concatenates activations; every arithmetic op is a kernel.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle
from .embedding import EmbeddingFeatures, SparseAdam, SparseTable
from .feature_config import FEATUREID_TO_SLOT, GATE_FEATURE_LIST, SlotLayout
from .layers import Dense, InteractingLayer, _DenseFn
from .models import SharedInputDense, _ActFn
from .params import FlatBlock, glorot_uniform_, grads_contiguous
from .towers import _BCEFn, _MixFn, _rows, gated, glorot_normal_

RELU, SIGMOID = 1, 2


def relu(x):
    return _ActFn.apply(x, RELU)


# ============================================================================================
# autograd wrappers of the front-end kernels
# ============================================================================================
class _GatherColsFn(torch.autograd.Function):
    """out[b, j] = src[b, cols[j]] (rs_gather_columns); backward scatter-adds (atomic: a column
    named twice in a plan receives both gradients, as TF's slice + concat gradient does)."""

    @staticmethod
    def forward(ctx, src, cols):
        src = _rows(src)
        B = src.shape[0]
        n = cols.numel()
        out = torch.empty(B, n, device=src.device)
        call("rs_gather_columns", stream_handle(), ptr(src), src.stride(0), B, ptr(cols), n,
             ptr(out), n)
        ctx.save_for_backward(cols)
        ctx.src_shape = src.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        (cols,) = ctx.saved_tensors
        B, S = ctx.src_shape
        dsrc = torch.zeros(B, S, device=dout.device)
        dout = dout.contiguous()
        call("rs_scatter_add_columns", stream_handle(), ptr(dout), dout.stride(0), B, ptr(cols),
             cols.numel(), ptr(dsrc), S)
        return dsrc, None


def gather_columns(src, cols):
    return _GatherColsFn.apply(src, cols)


def segment_mean(x, seg, F):
    """Per-field mean (no gradient: the SENet squeeze is under tf.stop_gradient,
    model_init.py:28)."""
    x = _rows(x).detach()
    out = torch.empty(x.shape[0], F, device=x.device)
    call("rs_segment_mean", stream_handle(), ptr(x), x.stride(0), x.shape[0], ptr(seg), F, ptr(out), F)
    return out


class _FieldScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s, seg, colfield, alpha):
        x, s = _rows(x), _rows(s)
        B, C = x.shape
        y = torch.empty(B, C, device=x.device)
        call("rs_field_scale_fwd", stream_handle(), ptr(x), x.stride(0), B, ptr(colfield), C, ptr(s),
             s.stride(0), float(alpha), ptr(y), C)
        ctx.save_for_backward(x, s, seg)
        ctx.alpha = float(alpha)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, s, seg = ctx.saved_tensors
        B, C = x.shape
        F = s.shape[1]
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ds = torch.empty(B, F, device=x.device) if ctx.needs_input_grad[1] else None
        if dx is None and ds is None:
            return None, None, None, None, None
        call("rs_field_scale_bwd", stream_handle(), ptr(dy), C, ptr(x), x.stride(0), B, ptr(seg), F,
             ptr(s), s.stride(0), ctx.alpha, ptr(dx), C, 0, ptr(ds), F)
        return dx, ds, None, None, None


class _FieldLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, bias, seg, colfield, F, O):
        x = _rows(x)
        B, C = x.shape
        y = torch.empty(B, F * O, device=x.device)
        call("rs_field_linear_fwd", stream_handle(), ptr(x), x.stride(0), B, ptr(seg), F, O, ptr(W),
             ptr(bias), ptr(y), F * O)
        ctx.save_for_backward(x, W, bias, seg, colfield)
        ctx.cfg = (F, O)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, bias, seg, colfield = ctx.saved_tensors
        F, O = ctx.cfg
        B, C = x.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ws_n = int(_lib.load().rs_field_linear_workspace_floats(B, C, F, O))
        ws = torch.empty(max(ws_n, 1), device=x.device)
        block = grads_contiguous((W, bias))
        dp = block if block is not None else torch.empty(W.numel() + bias.numel(), device=x.device)
        call("rs_field_linear_bwd", stream_handle(), ptr(dy), F * O, ptr(x), x.stride(0), B, ptr(seg),
             ptr(colfield), C, F, O, ptr(W), ptr(dx), C, 0, ptr(dp), dp.data_ptr() + 4 * W.numel(),
             1 if block is not None else 0, ptr(ws), ws_n)
        if block is not None:
            return dx, None, None, None, None, None, None
        return dx, dp[:W.numel()].view(W.shape), dp[W.numel():].view(bias.shape), None, None, None, None


class FieldLinear(nn.Module):
    """F per-field Keras Dense(O) maps (model_init.py:44-46) over the [B, C] concatenation of the
    fields (field f = columns [seg[f], seg[f+1])).  W [C, O] packs the fields' kernels
    (glorot_uniform with fan_in = that field's width), bias [F, O] (zeros)."""

    def __init__(self, widths: Sequence[int], units: int = 8, seed=0, device=None):
        super().__init__()
        dev = torch.device(device or "cuda")
        self.widths = [int(w) for w in widths]
        self.F, self.O = len(self.widths), int(units)
        self.C = sum(self.widths)
        seg = np.concatenate([[0], np.cumsum(self.widths)]).astype(np.int32)
        self.seg = torch.from_numpy(seg).to(dev)
        self.colfield = torch.from_numpy(np.repeat(np.arange(self.F), self.widths).astype(np.int32)).to(dev)
        blk = FlatBlock([(self.C, self.O), (self.F, self.O)], dev)
        self.kernel, self.bias = blk.params()
        gen = torch.Generator().manual_seed(seed)
        for f, w in enumerate(self.widths):
            t = torch.empty(w, self.O)
            glorot_uniform_(t, w, self.O, gen)
            with torch.no_grad():
                self.kernel[int(seg[f]):int(seg[f + 1])].copy_(t)

    def field_kernel(self, f):
        return self.kernel[int(self.seg[f]):int(self.seg[f + 1])]

    def forward(self, x):
        return _FieldLinearFn.apply(x, self.kernel, self.bias, self.seg, self.colfield, self.F, self.O)


class _CanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, p):
        r, p = _rows(r), _rows(p)
        B = r.shape[0]
        out = torch.empty(B, 4, device=r.device)
        h = torch.empty(B, 6, device=r.device)
        call("rs_can_fwd", stream_handle(), ptr(r), r.stride(0), ptr(p), p.stride(0), B, ptr(out), 4,
             ptr(h))
        ctx.save_for_backward(r, p, h, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        r, p, h, out = ctx.saved_tensors
        B = r.shape[0]
        dout = dout.contiguous()
        dr = torch.empty(B, 8, device=r.device)
        dp = torch.empty(B, 82, device=r.device)
        call("rs_can_bwd", stream_handle(), ptr(dout), 4, ptr(out), 4, ptr(r), r.stride(0), ptr(p),
             p.stride(0), ptr(h), B, ptr(dr), 8, 0, ptr(dp), 82)
        return dr, dp


def can_block(r, p):
    """CAN per-sample matmuls (model_init.py:90-98, 150-154): relu(relu(r W1 + b1) W2 + b2)."""
    return _CanFn.apply(r, p)


def clipped_cross_entropy(y_true, s):
    """cross_entropy (base_model.py:7-12) of tf.clip_by_value(s, 1e-6, 1.0) (model_init.py:158);
    the clip's gradient is zero outside [1e-6, 1] (rs_bce_clip_loss)."""
    return _BCEFn.apply(s, y_true, 1e-6, 1.0, 1e-6)


def clip_output(s):
    """tf.clip_by_value(s, 1e-6, 1.0) for inference (no gradient)."""
    s = _rows(s).detach()
    M, T = s.shape
    p = torch.empty_like(s)
    zeros = torch.zeros_like(s)
    call("rs_bce_clip_loss", stream_handle(), ptr(s), ptr(zeros), M, T, 1e-6, 1.0, 1e-6, None, ptr(p),
         None, None)
    return p


# ============================================================================================
# H2 + H12: rank/ctr
# ============================================================================================
@dataclass
class RankCtrConfig:
    bucket_size: int = 265_000        # category_column(bucket_size=265000), base_model.py:206
    lr_dense: float = 5e-5            # base_model.py:192
    lr_sparse: float = 5e-5           # base_model.py:163
    senet_reduction: int = 4          # model_init.py:27
    field_units: int = 8              # emb_linear_map Dense(8), :45
    il_dropout: float = 0.2           # :53-58
    ppnet_units: Sequence[int] = (256, 64, 8, 256, 64, 8, 32, 16)   # :65-69
    deep_units: Sequence[int] = (32, 16)                              # :73
    num_experts: int = 3                                              # :102
    expert_units: Sequence[int] = (512, 256)                          # :103
    gate_units: Sequence[int] = (256, 32)                             # :119
    tower_units: Sequence[int] = (64, 8)                              # :136
    can_units: int = 8 * 6 + 6 + 6 * 4 + 4                            # :91
    task_names: Sequence[str] = ("video_id_rank_hp_ctr_addfeasetwo_click",
                                 "video_id_rank_hp_ctr_addfeasetwo_effect_click")   # :138
    gate_feature_list: Sequence[str] = field(default_factory=lambda: list(GATE_FEATURE_LIST))


class RankCtrFrontEnd(nn.Module):
    """BaseModel's input layer on the device.  Every sparse feature id (sorted, base_model.py:
    70-73) is one VarLen field of an EmbeddingFeatures over ONE table: each distinct FeatureSlot
    (feature id, or the slot featureid_to_slot maps it to) owns `bucket_size` rows of width
    max_embed_size, so feature ids mapped to one slot share its rows (base_model.py:89-102)."""

    def __init__(self, layout: SlotLayout, cfg: RankCtrConfig, device=None, seed=0,
                 max_touched=None):
        super().__init__()
        dev = torch.device(device or "cuda")
        self.layout, self.cfg = layout, cfg
        self.features = list(layout.sparse_slots)
        self.table_slot = [FEATUREID_TO_SLOT.get(f, f) for f in self.features]
        regions = sorted(set(self.table_slot))
        self.region = {s: i for i, s in enumerate(regions)}
        D = layout.max_embed_size
        self.table = SparseTable(len(regions) * cfg.bucket_size, D, SparseAdam(cfg.lr_sparse),
                                 device=dev, seed=seed, max_touched=max_touched)
        self.embedding = EmbeddingFeatures(
            self.table, [cfg.bucket_size] * len(self.features),
            row_base=[self.region[s] * cfg.bucket_size for s in self.table_slot], combiner="mean")
        D = layout.max_embed_size
        i32 = dict(dtype=torch.int32, device=dev)
        si = layout.structure_intervals()
        self.struct_widths = [b - a for _, a, b in si]
        self.struct_cols = torch.tensor(layout.column_plan(si), **i32)
        self.gate_cols = torch.tensor(layout.column_plan(layout.gate_intervals(cfg.gate_feature_list)), **i32)
        self.bias_cols = {k: torch.tensor(layout.column_plan(v), **i32)
                          for k, v in layout.bias_intervals().items()}
        self.width = len(self.features) * D

    def forward(self, ids, offsets):
        """ids int64 [nnz], offsets int32 [B * n_features + 1] (feature-major within a sample):
        -> (structure [B, 2500], gate [B, G], {bias_type: [B, w]})."""
        emb = self.embedding(ids, offsets)                               # [B, F, D]
        flat = emb.reshape(emb.shape[0], -1)
        struct = gather_columns(flat, self.struct_cols)                   # emb_structure_input
        gate = gather_columns(flat, self.gate_cols)                       # emb_gate_input
        bias = {k: gather_columns(flat, c) for k, c in self.bias_cols.items()}   # emb_bias_input
        return struct, gate, bias


class RankCtrModel(nn.Module):
    """rank/ctr Model (model_init.py:12-167) over RankCtrFrontEnd."""

    def __init__(self, model_config: dict, cfg: RankCtrConfig | None = None, device=None, seed=0,
                 max_touched=None):
        super().__init__()
        self.cfg = cfg = cfg or RankCtrConfig()
        dev = torch.device(device or "cuda")
        self.layout = layout = SlotLayout.from_model_config(model_config)
        self.front = RankCtrFrontEnd(layout, cfg, device=dev, seed=seed, max_touched=max_touched)
        fe = self.front
        widths = fe.struct_widths
        Fs, C = len(widths), sum(widths)
        self.n_struct, self.struct_dim = Fs, C
        seg = np.concatenate([[0], np.cumsum(widths)]).astype(np.int32)
        self.seg = torch.from_numpy(seg).to(dev)
        self.colfield = torch.from_numpy(np.repeat(np.arange(Fs), widths).astype(np.int32)).to(dev)
        # SENet (:26-34): Dense(Fs // 4, relu) -> 2 * Dense(Fs, sigmoid)
        self.senet_sq = Dense(Fs // cfg.senet_reduction, "relu", seed=seed + 1, device=dev)
        self.senet_sq.build((1, Fs), device=dev)
        self.senet_ex = Dense(Fs, "sigmoid", seed=seed + 2, device=dev)
        self.senet_ex.build((1, Fs // cfg.senet_reduction), device=dev)
        # per-field Dense(8) (:43-46) -> InteractingLayer(1, 8, 2, dropout .2, res) (:53-58)
        self.field_map = FieldLinear(widths, cfg.field_units, seed=seed + 3, device=dev)
        self.interact = InteractingLayer(1, cfg.field_units, 2, use_dropout=True,
                                         dropout_rate=cfg.il_dropout, use_res=True, seed=seed + 4,
                                         device=dev)
        self.interact.build((1, Fs, cfg.field_units), device=dev)
        # ppnet gate 2 * Dense(704, sigmoid) on the ppnet bias group (:62-69)
        P = fe.bias_cols["ppnet"].numel()
        self.ppnet = Dense(sum(cfg.ppnet_units), "sigmoid", seed=seed + 5, device=dev)
        self.ppnet.build((1, P), device=dev)
        # deep Dense(32) -> gate -> relu -> Dense(16) -> gate -> relu (:73-78)
        self.deep = nn.ModuleList()
        d_in = C
        for i, u in enumerate(cfg.deep_units):
            layer = Dense(u, None, seed=seed + 10 + i, device=dev, name=f"dnn_{i}")
            layer.build((1, d_in), device=dev)
            self.deep.append(layer)
            d_in = u
        mu = fe.bias_cols["multiply_user"].numel()
        self.result_dim = R = cfg.deep_units[-1] + Fs * cfg.field_units + mu        # :89
        # CAN Dense(82) on the can bias group (:91-98)
        self.can = Dense(cfg.can_units, None, seed=seed + 20, device=dev)
        self.can.build((1, fe.bias_cols["can"].numel()), device=dev)
        # MMoE (:100-132): every layer reading `result` with relu is ONE GEMM (3 experts' first
        # layers + 2 gates' first layers); every first ppnet gate layer reads gate_input (one GEMM)
        NE, EU, GU = cfg.num_experts, list(cfg.expert_units), list(cfg.gate_units)
        self.first = SharedInputDense([EU[0]] * NE + [GU[0]] * 2, "relu", seed=seed + 30, device=dev)
        self.first.build((1, R), device=dev)
        G = fe.gate_cols.numel()
        self.pp1 = SharedInputDense([u for _ in range(NE) for u in EU], "relu", seed=seed + 40,
                                    device=dev)
        self.pp1.build((1, G), device=dev)
        self.pp2 = nn.ModuleList()
        self.exp_rest = nn.ModuleList()
        for i in range(NE):
            for j, u in enumerate(EU):
                g2 = Dense(u, "sigmoid", seed=seed + 50 + 10 * i + j, device=dev)
                g2.build((1, u), device=dev)
                self.pp2.append(g2)
                if j > 0:
                    e = Dense(u, "relu", seed=seed + 80 + 10 * i + j, device=dev)
                    e.build((1, EU[j - 1]), device=dev)
                    self.exp_rest.append(e)
        self.gate_l2 = nn.ModuleList()
        self.gate_out = nn.ModuleList()
        for t in range(2):
            g = Dense(GU[1], "relu", seed=seed + 110 + t, device=dev)
            g.build((1, GU[0]), device=dev)
            o = Dense(NE, None, seed=seed + 120 + t, device=dev)   # softmax inside rs_gate_mix
            o.build((1, GU[1]), device=dev)
            self.gate_l2.append(g)
            self.gate_out.append(o)
        self.sel = torch.arange(NE, dtype=torch.int32, device=dev).repeat(2)
        # task towers 256 -> 64 -> 8 (+ CAN 4) -> 1 (:134-160)
        self.towers = nn.ModuleList()
        self.outputs = nn.ModuleList()
        for t in range(2):
            layers = nn.ModuleList()
            d_in = EU[-1]
            for j, u in enumerate(cfg.tower_units):
                layer = Dense(u, None, seed=seed + 130 + 10 * t + j, device=dev, name=f"task{t}_dnn2_{j}")
                layer.build((1, d_in), device=dev)
                layers.append(layer)
                d_in = u
            self.towers.append(layers)
            out = Dense(1, "sigmoid", seed=seed + 150 + t, device=dev)
            out.build((1, cfg.tower_units[-1] + 4), device=dev)
            self.outputs.append(out)

    def tables(self):
        return [self.front.table]

    def regularizers(self):
        """L1L2(1e-5, 1e-5) on dnn_0/1 (:75) and task{i}_dnn2_{j} (:145)."""
        out = [(l.kernel, 1e-5, 1e-5) for l in self.deep]
        for layers in self.towers:
            out += [(l.kernel, 1e-5, 1e-5) for l in layers]
        return out

    def forward(self, ids, offsets):
        cfg, fe = self.cfg, self.front
        struct, gate_input, bias = fe(ids, offsets)
        B = struct.shape[0]
        # SENet over the stop-gradient field means (:21-40)
        sq = segment_mean(struct, self.seg, self.n_struct)
        s = self.senet_ex(self.senet_sq(sq))
        rew = _FieldScaleFn.apply(struct, s, self.seg, self.colfield, 2.0)        # [B, 2500]
        # per-field Dense(8) -> IL -> flatten (:43-60)
        auto_in = self.field_map(rew).reshape(B, self.n_struct, cfg.field_units)
        auto = self.interact(auto_in).reshape(B, -1)
        # ppnet gates (:62-69)
        pp = self.ppnet(bias["ppnet"])
        gl, o = [], 0
        for u in cfg.ppnet_units:
            gl.append(pp[:, o:o + u])
            o += u
        # deep (:71-78)
        deep = rew
        for i, layer in enumerate(self.deep):
            deep = relu(gated(layer(deep), gl[i + 6], 2.0))
        # multiply (:80-84)
        mult = relu(gated(bias["multiply_user"], bias["multiply_item"], 1.0))
        result = torch.cat([deep, auto, mult], dim=1)                             # :87
        # CAN parameters (:90-96)
        can_p = self.can(bias["can"])
        # MMoE (:98-132)
        NE, EU = cfg.num_experts, list(cfg.expert_units)
        firsts = self.first(result)
        pp1 = self.pp1(gate_input)
        experts, k = [], 0
        for i in range(NE):
            ex = None
            for j, u in enumerate(EU):
                g = self.pp2[i * len(EU) + j](pp1[i * len(EU) + j])             # 2 * sigmoid(.)
                ex = firsts[i] if j == 0 else self.exp_rest[k](ex)
                if j > 0:
                    k += 1
                ex = gated(ex, g, 2.0)                                            # tf.multiply
            experts.append(ex)
        gates = [self.gate_out[t](self.gate_l2[t](firsts[NE + t])) for t in range(2)]
        Z = torch.cat(experts + gates, dim=1)
        mm = _MixFn.apply(Z, self.sel, NE, EU[-1], 2, NE, 0)                       # softmax mix
        outs = []
        for t in range(2):
            r = mm[:, t * EU[-1]:(t + 1) * EU[-1]]
            r = relu(gated(r, gl[t * 3], 2.0))                                     # j == 0 (:140-142)
            for j, layer in enumerate(self.towers[t]):
                r = relu(gated(layer(r), gl[t * 3 + j + 1], 2.0))                  # :143-146
            can = can_block(r, can_p)                                              # :147-155
            r = torch.cat([r, can], dim=1)
            outs.append(self.outputs[t](r))                                        # Dense(1, sigmoid)
        return outs

    def loss(self, ids, offsets, labels):
        """The two cross_entropy losses (base_model.py:180-183), summed by Keras; labels [B, 2]."""
        outs = self.forward(ids, offsets)
        self.last_outputs = [o.detach() for o in outs]
        total = None
        for t, o in enumerate(outs):
            l = clipped_cross_entropy(labels[:, t:t + 1].contiguous(), o)
            total = l if total is None else total + l
        return total

    def predict(self, ids, offsets):
        """{task_name: clip(output, 1e-6, 1)} (:158-161)."""
        outs = self.forward(ids, offsets)
        return {n: clip_output(o) for n, o in zip(self.cfg.task_names, outs)}


# ============================================================================================
# H13: rank/finish FMLayer + DeepFM
# ============================================================================================
class _FMProjFn(torch.autograd.Function):
    """0.5 * sum((x V)^2 - x^2 V^2) + lin (lin = the Dense(1) linear term, [B, 1])."""

    @staticmethod
    def forward(ctx, x, V, lin):
        x = _rows(x)
        B, K = x.shape
        N = V.shape[1]
        lin = lin.reshape(B).contiguous()
        y = torch.empty(B, device=x.device)
        xv = torch.empty(B, N, device=x.device)
        call("rs_fm_proj_fwd", stream_handle(), ptr(x), x.stride(0), B, K, N, ptr(V), ptr(lin), ptr(y),
             ptr(xv))
        ctx.save_for_backward(x, V, xv)
        return y.reshape(B, 1)

    @staticmethod
    def backward(ctx, dy):
        x, V, xv = ctx.saved_tensors
        B, K = x.shape
        N = V.shape[1]
        dy = dy.reshape(B).contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ws_n = int(_lib.load().rs_fm_proj_workspace_floats(B, K, N))
        ws = torch.empty(max(ws_n, 1), device=x.device)
        dV = torch.empty_like(V)
        call("rs_fm_proj_bwd", stream_handle(), ptr(dy), ptr(x), x.stride(0), B, K, N, ptr(V), ptr(xv),
             ptr(dx), K, 0, ptr(dV), 0, ptr(ws), ws_n)
        return dx, dV, dy.reshape(B, 1)


class FMLayer(nn.Module):
    """rank/finish FMLayer(Dense) (videodnn.py:23-52): fm_matrix [D, 8] (GlorotNormal) and a
    Dense(1) linear term 'deeepfmlinear'; call(x) = 0.5 * sum((x V)^2 - x^2 V^2, axis=1) +
    Dense(1)(x) -> [B, 1].  (The staytime field-FM of staytime/layer.py:83-116 is
    towers.FMLayer.)"""

    def __init__(self, seed=1024, device=None, units=8):
        super().__init__()
        self.seed, self.units = seed, int(units)
        self._device = device
        self.built = False

    def build(self, input_shape, device=None):
        D = int(input_shape[-1])
        dev = device or self._device or torch.device("cuda")
        gen = torch.Generator().manual_seed(self.seed)
        V = torch.empty(D, self.units)
        glorot_normal_(V, D, self.units, gen)
        self.fm_matrix = nn.Parameter(V.to(dev))
        self.linear = Dense(1, None, seed=self.seed + 1, device=dev, name="deeepfmlinear")
        self.linear.build((1, D), device=dev)
        self.built = True

    def forward(self, inputs):
        if not self.built:
            self.build(tuple(inputs.shape), device=inputs.device)
        # tf.math.add(high_order_result, linear_result): the add is fused into the FM kernel
        return _FMProjFn.apply(inputs, self.fm_matrix, self.linear(inputs))


@dataclass
class DeepFMConfig:
    general_slots: Sequence[str] = ("3371", "3367", "3377", "2599", "2148", "2153", "2162", "2165",
                                    "2169", "2123", "2125", "2127", "2128", "2130", "2131", "2137",
                                    "2142", "2144", "2149", "2152", "2154", "2156", "1574", "1575",
                                    "1576", "1577", "1582", "1589", "1590", "1591", "1592", "1593",
                                    "1594", "1614", "1616", "1624", "1625", "1632", "1736", "1737",
                                    "1738", "1744", "1745", "1749", "2044", "2040", "2041", "2043",
                                    "2045", "2047", "2048", "2049", "2050", "2051", "2052")  # :73-78
    bias_slots: Sequence[str] = ("3051", "1570", "2039", "2544", "1568", "3376", "3365", "3369",
                                 "2597")                                                     # :72
    emb_dim: int = 32               # embedding_column(dimension=32), :59
    bucket_size: int = 25_600       # :56
    dnn_hidden_units: Sequence[int] = (64, 32)   # DEEPFM default, :172
    lr_dense: float = 1e-3          # rank/finish/model.py:37
    lr_sparse: float = 1e-3         # :62
    task_name: str = "video_id_rank_finish_nb_lr_rongh_bundle"


class DeepFM(nn.Module):
    """rank/finish DEEPFM (videodnn.py:69-196).  Slots (config.SLOTS is not in the reference;
    pinned: general + bias slots, sorted as the reference sorts emb_input_shapes) each look up
    a mean-pooled [B, 32] row; general = concat(slot[:, 0:16] over the 55 general slots in
    sorted order, then emb_1568[:, 16:32]) [B, 56*16]; bias = concat(slot[:, 0:16] over bias slots)
    [B, 144]; FMLayer(general); deep: relu(Dense(64)) then, per further unit u, relu(Dense(u)(x *
    2 sigmoid(Dense(prev)(relu(Dense(prev)(bias)))))); final x * 2 sigmoid(Dense(u)(relu(
    Dense(u)(bias)))); output Dense(1, sigmoid) on [x, fm]."""

    def __init__(self, cfg: DeepFMConfig | None = None, device=None, seed=0, max_touched=None):
        super().__init__()
        self.cfg = cfg = cfg or DeepFMConfig()
        dev = torch.device(device or "cuda")
        self.slots = sorted(set(cfg.general_slots) | set(cfg.bias_slots))
        S = len(self.slots)
        self.table = SparseTable(S * cfg.bucket_size, cfg.emb_dim, SparseAdam(cfg.lr_sparse), device=dev,
                                 seed=seed, max_touched=max_touched)
        self.embedding = EmbeddingFeatures(self.table, [cfg.bucket_size] * S, combiner="mean")
        pos = {s: i for i, s in enumerate(self.slots)}
        E = cfg.emb_dim
        gen_cols = [pos[s] * E + c for s in self.slots if s in set(cfg.general_slots) for c in range(16)]
        gen_cols += [pos["1568"] * E + c for c in range(16, 32)]                      # :87
        bias_cols = [pos[s] * E + c for s in self.slots if s in set(cfg.bias_slots) for c in range(16)]
        i32 = dict(dtype=torch.int32, device=dev)
        self.gen_cols = torch.tensor(gen_cols, **i32)
        self.bias_cols = torch.tensor(bias_cols, **i32)
        Dg, Db = len(gen_cols), len(bias_cols)
        self.fm = FMLayer(seed=seed + 1, device=dev)
        self.fm.build((1, Dg), device=dev)
        H = list(cfg.dnn_hidden_units)
        self.dnn = nn.ModuleList()
        self.b_one = nn.ModuleList()
        self.b_two = nn.ModuleList()
        d_in = Dg
        for i, u in enumerate(H):
            layer = Dense(u, "relu", seed=seed + 10 + i, device=dev, name=f"dnn_{i}")
            layer.build((1, d_in), device=dev)
            self.dnn.append(layer)
            d_in = u
        # bias gates: one pair per hidden unit after the first (width = previous unit), plus the
        # final pair (width = last unit) -- :104-125
        for u in H[:-1] + [H[-1]]:
            one = Dense(u, "relu", seed=seed + 20 + len(self.b_one), device=dev)
            one.build((1, Db), device=dev)
            two = Dense(u, "sigmoid", seed=seed + 30 + len(self.b_two), device=dev)
            two.build((1, u), device=dev)
            self.b_one.append(one)
            self.b_two.append(two)
        self.pred = Dense(1, "sigmoid", seed=seed + 40, device=dev, name="pred")
        self.pred.build((1, H[-1] + 1), device=dev)

    def tables(self):
        return [self.table]

    def regularizers(self):
        """L1L2(1e-5, 1e-5) on dnn_i and bais_dnn_{one,two}_i kernels (:98-118)."""
        return [(l.kernel, 1e-5, 1e-5) for l in list(self.dnn) + list(self.b_one) + list(self.b_two)]

    def forward(self, ids, offsets=None):
        """ids [B, n_slots] (one id per slot) or VarLen (ids, offsets) over the sorted slots."""
        emb = self.embedding(ids, offsets)
        flat = emb.reshape(emb.shape[0], -1)
        general = gather_columns(flat, self.gen_cols)
        bias = gather_columns(flat, self.bias_cols)
        fm = self.fm(general)                                                     # :90-91
        x = general
        for i, layer in enumerate(self.dnn):
            if i == 0:
                x = layer(x)                                                      # :101-102
            else:
                g = self.b_two[i - 1](self.b_one[i - 1](bias))
                x = layer(gated(x, g, 2.0))                                       # :110-112
        g = self.b_two[-1](self.b_one[-1](bias))
        x = gated(x, g, 2.0)                                                      # :125
        return self.pred(torch.cat([x, fm], dim=1))                               # :126-127

    def loss(self, ids, offsets, labels):
        """cross_entropy (rank/finish/model.py:19-25) on the (unclipped) sigmoid output."""
        from .towers import cross_entropy_sum
        return cross_entropy_sum(labels, self.forward(ids, offsets))
