"""AutoInt CTR model (autoint:11-60 on the rank/ctr BaseModel front end) and its training step.

Two entry points share the same kernels:
  * ``AutoInt`` — an nn.Module with the reference's structure (embedding concat -> InteractingLayer
    -> flatten; deep MultiLayerDense on the flattened embeddings; concat [deep, autoint];
    logits MultiLayerDense; clip_by_value(1e-6, 1)); ``forward`` is autograd-composable and
    ``run()`` returns {"train": model, "predict": model} like autoint:58-60.
  * ``AutoIntTrainer`` — the fused training step (what tensornet's model.fit runs per batch):
    forward, cross_entropy, backward, dense Adam and sparse Adam, issued as ~20 launches into
    preallocated buffers (no allocation, no host sync) and captured into one HIP graph.
    Activations are laid out so that concats are free: the IL writes its flattened output and
    the deep tower its last layer straight into the [B, D + F*U] concat buffer (autoint:44).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle
from .dist import capture_error_mode
from .embedding import EmbeddingFeatures, SparseAdam, SparseTable
from .layers import ACTIVATIONS, InteractingLayer, MultiLayerDense
from .params import ParamArena


@dataclass
class AutoIntConfig:
    """model_config['model_param'] of autoint:30-50 plus the front end.  The shipped
    rank/ctr/model_parameter.json has no 'model_param' block, so defaults are the pinned config-2
    values (SURVEY §8c decision 3): IL(3, 16, 2, res), mlp [32, 16] relu, logits [1] sigmoid."""
    num_fields: int = 26
    embed_dim: int = 16
    vocab_per_field: int = 100_000
    layer_num: int = 3
    unit_num: int = 16
    head_num: int = 2
    use_dropout: bool = False
    dropout_rate: float = 0.0
    use_res: bool = True
    ln_eps: float = 1e-14
    mlp_hidden: Sequence[int] = (32, 16)
    mlp_activation: str = "relu"
    logits_hidden: Sequence[int] = (1,)
    logits_activation: str = "sigmoid"
    lr_dense: float = 5e-5    # rank/ctr/base_model.py:192
    lr_sparse: float = 5e-5   # rank/ctr/base_model.py:163
    hash_mode: str = "mod"
    combiner: str = "mean"    # embedding_column(..., combiner='mean') base_model.py:211
    # "f32" (the reference's dtype) or "bf16": config 2's bf16 compute mode (BASELINE.json
    # configs[1]) -- the IL and MLP-head GEMMs take bf16 operands with fp32 accumulation, master
    # weights / tables / optimizer state stay fp32 (rs_set_math_mode, include/recsys_amd.h)
    compute_dtype: str = "f32"

    @staticmethod
    def from_model_config(model_config: dict, **front) -> "AutoIntConfig":
        mp = model_config["model_param"]
        it, ml, lg = mp["interact"], mp["mlp"], mp["logits"]
        return AutoIntConfig(layer_num=it["layer_num"], unit_num=it["unit_num"],
                             head_num=it["head_num"], use_dropout=it["use_dropout"],
                             dropout_rate=it["dropout_rate"], use_res=it["use_res"],
                             mlp_hidden=tuple(ml["hidden_units"]), mlp_activation=ml["activation"],
                             logits_hidden=tuple(lg["hidden_units"]),
                             logits_activation=lg["activation"], **front)


class AutoInt(nn.Module):
    def __init__(self, cfg: AutoIntConfig | dict | None = None, device=None, seed: int = 0,
                 max_batch: int = 4096, world_size: int = 1):
        super().__init__()
        if isinstance(cfg, dict):
            cfg = AutoIntConfig.from_model_config(cfg)
        self.cfg = cfg = cfg or AutoIntConfig()
        dev = torch.device(device or "cuda")
        F, E, U = cfg.num_fields, cfg.embed_dim, cfg.unit_num
        self.table = SparseTable(F * cfg.vocab_per_field, E, SparseAdam(cfg.lr_sparse), device=dev,
                                 seed=seed, max_touched=max_batch * F * world_size)
        self.embedding = EmbeddingFeatures(self.table, [cfg.vocab_per_field] * F,
                                           combiner=cfg.combiner, hash_mode=cfg.hash_mode)
        self.interact = InteractingLayer(cfg.layer_num, U, cfg.head_num, cfg.use_dropout,
                                         cfg.dropout_rate, cfg.use_res, ln_epsilon=cfg.ln_eps,
                                         seed=seed + 1, device=dev)
        self.interact.build((1, F, E), device=dev)
        self.deep = MultiLayerDense(cfg.mlp_hidden, cfg.mlp_activation, seed=seed + 10, device=dev)
        d_in = F * E
        for layer in self.deep.layers:
            layer.build((1, d_in), device=dev)
            d_in = layer.units
        self.logits = MultiLayerDense(cfg.logits_hidden, cfg.logits_activation, seed=seed + 20,
                                      device=dev)
        d_in = cfg.mlp_hidden[-1] + F * U
        for layer in self.logits.layers:
            layer.build((1, d_in), device=dev)
            d_in = layer.units
        self.arena = ParamArena(self.parameters(), device=dev)

    # autograd-composable forward (autoint:18-56); returns the clipped prediction p
    def forward(self, ids: torch.Tensor, offsets: torch.Tensor | None = None) -> torch.Tensor:
        return self.dense_forward(self.embedding(ids, offsets))  # [B, F, E]  (autoint:22-26)

    def dense_forward(self, x0: torch.Tensor) -> torch.Tensor:
        """The dense sub_model over the field embeddings x0 [B, F, E] (export.autoint_sub_model)."""
        B = x0.shape[0]
        il = self.interact(x0).reshape(B, -1)                   # :30-36
        deep = self.deep(x0.reshape(B, -1))                     # :39-41
        result = torch.cat([deep, il], dim=1)                   # :44
        s = self.logits(result)                                 # :48-50
        return torch.clamp(s, 1e-6, 1.0)                        # :52

    def run(self):
        """autoint:58-60 / rank/ctr/base_model.py:169-201: {"train": model, "predict": model}."""
        return {"train": self, "predict": self}


def cross_entropy(y_true: torch.Tensor, y_pred: torch.Tensor, a: float = 1.0) -> torch.Tensor:
    """rank/ctr/base_model.py:7-12 (autograd form, for the composable path)."""
    y_true = y_true.to(torch.float32)
    loss = -y_true * torch.log(y_pred + 1e-6) - (a - y_true) * torch.log(1.0 - y_pred + 1e-6)
    return torch.mean(torch.sum(loss, dim=1), dim=0)


# the largest B x F for which the single-GPU step's sparse Adam walks the looked-up rows instead of
# sweeping the flag array (rows mode).  Same box, 200 steps (profiles/r04/final/rows_mode/): B = 512
# 0.0580 -> 0.0537 ms, 1024 0.0717 -> 0.0714, 2048 0.0972 -> 0.1041 (worse: the Zipf-hot rows'
# flag exchanges serialise), 4096 0.1523 -> 0.1689
ROWS_MODE_MAXN = 26 * 1024


class AutoIntTrainer:
    """Fused AutoInt train step over fixed-shape batches (ids int64 [B, F], labels fp32 [B, T]).

    Per step: lookup -> IL fwd -> deep fwd -> logits fwd -> clip+BCE (+ dloss) -> logits bwd ->
    deep bwd -> IL bwd (accumulating into the embedding gradient) -> sparse push ->
    [data-parallel exchange] -> dense Adam (one flat arena) -> sparse Adam (touched rows).
    ``capture()`` records the step into a torch.cuda.CUDAGraph (hipGraph); ``step()`` replays it.
    """

    def __init__(self, model: AutoInt, batch_size: int, process_group=None,
                 deterministic: bool = False, metrics=None, dp_world1: bool = False):
        """metrics: a metrics.CtrMetrics updated with (p, labels) inside every step (the Keras
        'acc' / AUC() / tn.metric.COPC() of rank/ctr/base_model.py:183-190; one more launch per
        step, captured with the rest), or one CtrMetrics per task for a multi-task head (task t
        reads column t of p and labels).  None (the benchmark) skips it.
        dp_world1: run the data-parallel step (exchange, rank-ordered merges) on a world-1 group
        too (tests: the RCCL path on a one-GPU box)."""
        self.model = m = model
        if metrics is not None and not isinstance(metrics, (list, tuple)):
            metrics = [metrics]
        self.metrics = list(metrics) if metrics is not None else None
        cfg = m.cfg
        self.B = B = int(batch_size)
        self.F, self.E, self.U = F, E, U = cfg.num_fields, cfg.embed_dim, cfg.unit_num
        self.L, self.H = cfg.layer_num, cfg.head_num
        dev = m.table.weight.device
        self.dev = dev
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.dp = self.world > 1 or (bool(dp_world1) and process_group is not None)
        f32 = dict(device=dev, dtype=torch.float32)
        self.deep_layers = list(m.deep.layers)
        self.logit_layers = list(m.logits.layers)
        self.D = D = cfg.mlp_hidden[-1]
        self.CW = CW = D + F * U
        self.T = self.logit_layers[-1].units
        if self.metrics is not None and len(self.metrics) != self.T:
            raise ValueError(f"metrics: one CtrMetrics per task ({self.T}), got {len(self.metrics)}")
        # static inputs
        self.ids = torch.zeros(B, F, device=dev, dtype=torch.int64)
        self.labels = torch.zeros(B, self.T, **f32)
        # activations
        self.x0 = torch.empty(B, F * E, **f32)
        self.rows = torch.empty(B * F, device=dev, dtype=torch.int32)
        self.xsave = torch.empty(max(self.L - 1, 1), B, F, U, **f32)
        self.cat = torch.empty(B, CW, **f32)
        self.h = [torch.empty(B, l.units, **f32) for l in self.deep_layers[:-1]]
        self.lh = [torch.empty(B, l.units, **f32) for l in self.logit_layers[:-1]]
        self.s = torch.empty(B, self.T, **f32)
        self.p = torch.empty(B, self.T, **f32)
        self.loss = torch.zeros(1, **f32)
        # gradients
        self.ds = torch.empty(B, self.T, **f32)
        self.dcat = torch.empty(B, CW, **f32)
        self.dh = [torch.empty_like(t) for t in self.h]
        self.dlh = [torch.empty_like(t) for t in self.lh]
        self.dx0 = torch.empty(B, F * E, **f32)
        lib = _lib.load()
        self.il_ws_n = int(lib.rs_il_bwd_workspace_floats(B, E, U))
        # the saved-attention pair (rs_il_fwd_gather_saved / rs_il_bwd_push_saved; 0 floats for
        # shapes without one): the forward's attention output + softmax stats per (iteration,
        # sample), so the backward skips the softmax re-run (config 2: 25 MB at B = 4096)
        self.asave_n = int(lib.rs_il_attn_save_floats(B, F, U, self.H, self.L))
        self.asave = torch.empty(max(self.asave_n, 1), **f32)
        ws_dense = max(int(lib.rs_dense_bwd_weight_workspace_floats(B, l.input_dim, l.units))
                       for l in self.deep_layers + self.logit_layers)
        self.dense_ws_n = ws_dense
        self.il_ws = torch.empty(self.il_ws_n, **f32)
        self.dense_ws = torch.empty(ws_dense, **f32)
        # dense optimizer state on the flat arena
        ar = m.arena
        self.adam_m = torch.zeros_like(ar.data)
        self.adam_v = torch.zeros_like(ar.data)
        self.step_count = torch.zeros(1, device=dev, dtype=torch.int64)
        il = m.interact
        self.il_dparams = ar.grad[self._offset(il.kernel):self._offset(il.kernel) +
                                  il.kernel.numel() + il.bias.numel() + il.gamma.numel() + il.beta.numel()]
        self.graph = None
        self.graph_opt = None
        self.pool_graphs = []
        if cfg.compute_dtype not in _lib.MATH_MODES:
            raise ValueError(f"compute_dtype must be one of {sorted(_lib.MATH_MODES)}")
        # the InteractingLayer kernel variant (rs_il_set_variant) is pinned at construction: the
        # plan below sizes the partial-row reduction from the variant's backward grid, and every
        # step / capture runs under the same variant (a later process-wide change cannot land the
        # step on a kernel with another grid)
        self.il_variant = {v: k for k, v in _lib.IL_VARIANTS.items()}[int(lib.rs_il_get_variant())]
        with _lib.il_variant(self.il_variant), _lib.math_mode(cfg.compute_dtype):
            self.head = self._plan_head()
        if cfg.compute_dtype == "bf16" and (self.head is None or self.F > 32 or E != 16 or
                                            U != 16 or self.H != 2 or
                                            (self.head["N1"], self.head["N2"]) != (32, 16)):
            raise ValueError("bf16 compute mode has kernels for the config-2 shape only (F <= 32, "
                             "E = U = 16, H = 2, fused head with mlp [32, 16])")
        # fused path: the IL backward pushes dL/dx0 straight into the table (scan-mode marks);
        # deterministic: dL/dx0 is stored and pushed by the sorted segmented sum instead (bitwise
        # reproducible embedding gradients; one more launch and a dx0 round trip)
        self.deterministic = bool(deterministic)
        self.push = self.head is not None and self.F <= 64 and not self.deterministic
        if self.deterministic:
            m.table.deterministic = True
            m.table.sorted_workspace(B * F)
        if self.push:
            m.table.mode = "scan"
        # data parallel, fused path: packed exchange (dist.exchange_packed) -- the dense partials
        # reduce into a send bucket that also carries the sparse record count, the touched rows
        # are packed into [row | grad] records; two all-gathers, then graph-captured rank-ordered
        # merges and a rank-ordered dense sum fused with Adam
        self.packed_dp = self.dp and self.push
        if self.packed_dp:
            n = m.arena.n
            self.dp_n = n
            self.dp_rs = E + 1
            self.dp_nmax = 0
            # exchange without a host read; RS_DP_SYNC=1 restores the count-sized exchange with
            # one host synchronisation per step (A/B)
            import os
            self.dp_sync_free = not os.environ.get("RS_DP_SYNC")
            if self.dp_sync_free:
                # ONE all-gather per step (dist.packed_layout): [dense grad | count | records],
                # cap = B x F records (one rank touches at most that many rows per step)
                from .dist import packed_layout
                self.dp_ld, self.dp_cap, self.dp_S = packed_layout(n, B * F, self.dp_rs)
                self.dp_buf = torch.zeros(self.dp_S, **f32)
                self.dp_send = self.dp_buf[:self.dp_ld]
                self.dp_recs = self.dp_buf[self.dp_ld:]
                self.dp_all = torch.zeros(self.world * self.dp_S, **f32)
                # RCCL: the all-gather is captured with the rest of the step, ONE graph per pool
                # batch (thread_local capture, dist.capture_error_mode); gloo collectives are host
                # calls and stay eager between a forward/backward and an optimizer graph
                # (RS_DP_SPLIT_GRAPH=1 forces that form on RCCL too)
                from .dist import uses_flat_all_gather
                self.dp_one_graph = (uses_flat_all_gather(process_group) and
                                     not os.environ.get("RS_DP_SPLIT_GRAPH"))
            else:
                self.dp_ld = ld = (n + 1 + 3) // 4 * 4
                self.dp_cap = B * F
                self.dp_send = torch.zeros(ld, **f32)
                self.dp_recv = torch.zeros(self.world * ld, **f32)
                self.dp_recs = torch.empty(self.dp_cap * self.dp_rs, **f32)
                self.dp_recs_all = torch.empty(self.world * self.dp_cap * self.dp_rs, **f32)
        elif self.dp:
            cap = m.table.touched_cap
            self.x_rows = torch.empty(cap, device=dev, dtype=torch.int32)
            self.x_grads = torch.empty(cap, E, **f32)
            self.x_count = torch.zeros(1, device=dev, dtype=torch.int32)

    @property
    def _one_graph(self) -> bool:
        """One captured graph per step: single-GPU, or DP whose collective can be captured."""
        return not self.dp or getattr(self, "dp_one_graph", False)

    def _offset(self, p: torch.Tensor) -> int:
        return (p.data_ptr() - self.model.arena.data.data_ptr()) // 4

    def _grad(self, p: torch.Tensor) -> int:
        return self.model.arena.grad.data_ptr() + 4 * self._offset(p)

    # ---------------------------------------------------------------------------------------
    def _plan_head(self):
        """Use the fused head kernel (rs_mlp_head_train) when the towers fit its instantiations:
        deep [N1] or [N1, N2], logits [T <= 4], parameters laid out [W1 b1 (W2 b2) W3 b3] in the
        arena right after the InteractingLayer's [W b gamma beta].  Otherwise the per-layer
        Dense entry points run (same math)."""
        supported = {(32, 16), (64, 32), (16, 0), (32, 0), (64, 0), (16, 16), (32, 32), (64, 16),
                     (64, 64)}
        deep, logit = self.deep_layers, self.logit_layers
        if len(deep) not in (1, 2) or len(logit) != 1 or logit[0].units > 4:
            return None
        N1 = deep[0].units
        N2 = deep[1].units if len(deep) == 2 else 0
        if (N1, N2) not in supported or (self.F * self.E) % 16 or (self.F * self.U) % 4:
            return None
        params = [deep[0].kernel, deep[0].bias] + ([deep[1].kernel, deep[1].bias] if N2 else []) + \
                 [logit[0].kernel, logit[0].bias]
        off = self._offset(params[0])
        o = off
        for p in params:
            if self._offset(p) != o:
                return None
            o += p.numel()
        il = self.model.interact
        il_off = self._offset(il.kernel)
        il_n = il.kernel.numel() + il.bias.numel() + il.gamma.numel() + il.beta.numel()
        if il_off + il_n > self.model.arena.n:
            return None
        lib = _lib.load()
        K0, S, T = self.F * self.E, self.F * self.U, logit[0].units
        npar = int(lib.rs_mlp_head_param_floats(K0, N1, N2, S, T))
        if npar != o - off:
            return None
        dev = self.dev
        # deferred dW1 (rs_mlp_head_train_dz): the head stores dz1 [B, N1] and the IL backward's
        # waves form dW1 = x0^T dz1 as rs_il_xt_splits(B) sample-range partial rows
        # (rs_il_bwd_push_saved_xt), instead of K0 x N1 partial floats per 16-sample head block
        # (57 KB x B / 16: 14.6 MB written and read back per B = 4096 step).  Needs a saved
        # backward that carries it (rs_il_bwd_xt_supported); RS_HEAD_W1_PARTIALS=1 keeps the
        # partial-row form (A/B runs)
        import os
        dz = (not os.environ.get("RS_HEAD_W1_PARTIALS") and self.asave_n > 0 and
              lib.rs_il_bwd_xt_supported(self.B, self.F, self.E, self.U, self.H, self.il_ws_n) > 0)
        w1n = K0 * N1 if dz else 0
        nws = (lib.rs_mlp_head_dz_workspace_floats if dz else lib.rs_mlp_head_workspace_floats)(
            self.B, K0, N1, N2, S, T)
        ws = torch.empty(int(nws), device=dev, dtype=torch.float32)
        xt = None
        if dz:
            ns = int(lib.rs_il_xt_splits(self.B))
            xt = dict(dz1=torch.zeros(self.B, N1, device=dev, dtype=torch.float32), splits=ns,
                      slab=torch.zeros(ns * K0 * N1, device=dev, dtype=torch.float32))
        return dict(N1=N1, N2=N2, T=T, K0=K0, S=S, off=off, npar=npar, ws=ws, xt=xt,
                    # the partial rows: [b1 ... b3 | loss] (deferred dW1) or [W1 b1 ... | loss]
                    w1n=w1n, pn=npar - w1n,
                    blocks=int(lib.rs_mlp_head_partial_blocks(self.B)),
                    il_off=il_off, il_n=il_n,
                    # the step's backward reads the forward's attention save when the shape
                    # has one (rs_il_bwd_push_saved / rs_il_bwd_saved): its kernels' grid
                    il_blocks=int((lib.rs_il_bwd_saved_partial_blocks if self.asave_n > 0
                                   else lib.rs_il_bwd_partial_blocks)(
                        self.B, self.F, self.E, self.U, self.H, self.il_ws_n)),
                    done=torch.zeros(288, device=dev, dtype=torch.int32))

    def _forward_backward_fused(self):
        """lookup + IL fwd (one launch for F <= 64) -> fused head (MLP fwd, clip+BCE, MLP bwd) ->
        IL bwd + sparse push: three launches; dense gradients stay as per-block partials until
        _reduce_dense."""
        m, hd = self.model, self.head
        B, F, E, U, L, H, D, CW = self.B, self.F, self.E, self.U, self.L, self.H, self.D, self.CW
        s = stream_handle()
        il, emb, t = m.interact, m.embedding, m.table
        drop = il.dropout_rate if il.use_dropout else 0.0
        if F > 64:  # the many-field IL kernels read x0 from the lookup
            call("rs_embedding_lookup_fwd", s, ptr(self.ids), None, B, F, ptr(emb.row_base),
                 ptr(emb.bucket), emb.hash_mode, emb.combiner, ptr(t.weight), t.rows, E,
                 ptr(self.x0), F * E, E, ptr(self.rows))
            call("rs_il_fwd", s, ptr(self.x0), B, F, E, U, H, L, ptr(il.kernel), ptr(il.bias),
                 ptr(il.gamma), ptr(il.beta), il.epsilon, int(il.use_res), drop, il.seed,
                 self.cat.data_ptr() + 4 * D, CW, ptr(self.xsave) if L > 1 else None)
        else:  # single-hot lookup + concat + IL forward in one launch (x0 and the hashed rows
            # are by-products for the head and the push)
            call("rs_il_fwd_gather_saved", s, ptr(self.ids), ptr(emb.row_base), ptr(emb.bucket),
                 emb.hash_mode, ptr(t.weight), t.rows, ptr(self.x0), ptr(self.rows), B, F, E, U,
                 H, L, ptr(il.kernel), ptr(il.bias), ptr(il.gamma), ptr(il.beta), il.epsilon,
                 int(il.use_res), drop, il.seed, self.cat.data_ptr() + 4 * D, CW,
                 ptr(self.xsave) if L > 1 else None, ptr(self.asave), self.asave_n)
        d = self.deep_layers
        lg = self.logit_layers[0]
        d2 = d[1] if hd["N2"] else None
        xt = hd["xt"]
        call("rs_mlp_head_train_dz" if xt else "rs_mlp_head_train", s, ptr(self.x0), F * E,
             self.cat.data_ptr() + 4 * D, CW, B,
             hd["K0"], hd["S"], hd["N1"], d[0].act, hd["N2"], d2.act if d2 is not None else 0,
             hd["T"], lg.act, ptr(d[0].kernel), ptr(d[0].bias),
             ptr(d2.kernel) if d2 is not None else None, ptr(d2.bias) if d2 is not None else None,
             ptr(lg.kernel), ptr(lg.bias), ptr(self.labels), 1e-6, 1.0, 1e-6, ptr(self.p),
             self.dcat.data_ptr() + 4 * D, CW, ptr(self.dx0), F * E, 0, ptr(hd["ws"]),
             hd["ws"].numel(), *((ptr(xt["dz1"]), hd["N1"]) if xt else ()))
        # the deferred dW1 rides on the IL backward (x0^T dz1 partial rows)
        xa = (ptr(self.x0), F * E, ptr(xt["dz1"]), hd["N1"], hd["K0"], hd["N1"],
              ptr(xt["slab"])) if xt else ()
        if self.push:
            # dL/dx0 = head share (dx0) + IL share, added straight into the table rows
            call("rs_il_bwd_push_saved_xt" if xt else "rs_il_bwd_push_saved", s, ptr(self.x0),
                 ptr(self.xsave) if L > 1 else None,
                 self.dcat.data_ptr() + 4 * D, CW, B, F, E, U, H, L, ptr(il.kernel), ptr(il.bias),
                 ptr(il.gamma), ptr(il.beta), il.epsilon, int(il.use_res), drop, il.seed,
                 ptr(self.dx0), ptr(self.rows), ptr(t.grad), ptr(t.flag), None, 0,
                 ptr(self.il_ws), self.il_ws_n, ptr(self.asave), self.asave_n, *xa)
            return
        # (F > 64: the forward above is the plain one, no save to read)
        saved = F <= 64 and self.asave_n > 0
        name, tail = ("rs_il_bwd_saved", (ptr(self.asave), self.asave_n)) if saved else ("rs_il_bwd", ())
        if xt:
            name, tail = "rs_il_bwd_saved_xt", tail + xa
        call(name, s, ptr(self.x0), ptr(self.xsave) if L > 1 else None,
             self.dcat.data_ptr() + 4 * D, CW, B, F, E, U, H, L, ptr(il.kernel), ptr(il.bias),
             ptr(il.gamma), ptr(il.beta), il.epsilon, int(il.use_res), drop, il.seed, ptr(self.dx0),
             1, None, 0, ptr(self.il_ws), self.il_ws_n, *tail)
        t.accumulate(self.rows, None, B, F, self.dx0, F * E, E, emb.combiner)

    def _scan_tail(self, table):
        """The table when its sparse optimizer can run inside the dense reduce + Adam launch
        (scan mode, sparse Adam; rs_partials_reduce_adam_scan), else None."""
        import os
        from .embedding import SparseAdam
        ok = (not os.environ.get("RS_NO_FUSED_TAIL")  # A/B switch (two launches)
              and getattr(table, "mode", None) == "scan" and isinstance(table.optimizer, SparseAdam)
              and not getattr(table, "deterministic", False) and hasattr(table, "m"))
        return table if ok else None

    def _reduce_dense(self, adam: bool, scan_table=None, scan_rows=None):
        """Sum the IL and head partials (fixed order) into the arena gradient and the loss; with
        adam, apply the dense Adam in the same launch (and, with scan_table, its sparse Adam)."""
        m, hd, cfg = self.model, self.head, self.model.cfg
        ar = m.arena
        # data parallel: the local gradient goes to the exchange bucket, not the arena
        g0 = self.dp_send.data_ptr() if self.packed_dp else ar.grad.data_ptr()
        pn, ho = hd["pn"], hd["off"] + hd["w1n"]  # partial-row columns and their arena offset
        segs = [
            (self.il_ws.data_ptr(), hd["il_n"], hd["il_blocks"], hd["il_n"], g0 + 4 * hd["il_off"],
             1.0, hd["il_off"]),
            (hd["ws"].data_ptr(), pn + 1, hd["blocks"], pn, g0 + 4 * ho, 1.0, ho),
            (hd["ws"].data_ptr() + 4 * pn, pn + 1, hd["blocks"], 1, self.loss.data_ptr(),
             1.0 / self.B, -1),
        ]
        xt = hd["xt"]
        if xt is not None:  # dW1's sample-range rows from the IL backward (rs_il_bwd_*_xt)
            w1 = hd["K0"] * hd["N1"]
            segs.insert(1, (xt["slab"].data_ptr(), w1, xt["splits"], w1, g0 + 4 * hd["off"], 1.0,
                            hd["off"]))
        _lib.partials_reduce_adam(stream_handle(), segs, ar.data, self.adam_m, self.adam_v,
                                  self.step_count, hd["done"], cfg.lr_dense, 0.9, 0.999, 1e-8,
                                  1.0 / self.world, adam, scan_table=scan_table,
                                  scan_rows=scan_rows)

    def _forward_backward(self):
        # math mode of the step; dropout seeds offset by the device step counter (fresh masks on
        # every graph replay, rs_set_seed_offset)
        with _lib.math_mode(self.model.cfg.compute_dtype), _lib.seed_offset(self.step_count), \
                _lib.il_variant(self.il_variant):
            self._forward_backward_modal()

    def _forward_backward_modal(self):
        self._forward_backward_core()
        if self.metrics is not None:
            for t, mt in enumerate(self.metrics):  # column t of the [B, T] outputs / labels
                mt.update(self.p[:, t:t + 1], self.labels[:, t:t + 1])

    def _forward_backward_core(self):
        if self.head is not None:
            self._forward_backward_fused()
            if self.dp:
                self._reduce_dense(adam=False)
            if self.packed_dp:
                t = self.model.table
                call("rs_sparse_pack_scan", stream_handle(), ptr(t.grad), ptr(t.flag), t.rows,
                     t.dim, ptr(self.dp_recs), self.dp_send.data_ptr() + 4 * self.dp_n,
                     self.dp_cap)
            return
        m, cfg = self.model, self.model.cfg
        B, F, E, U, L, H, D, CW = self.B, self.F, self.E, self.U, self.L, self.H, self.D, self.CW
        s = stream_handle()
        il = m.interact
        emb = m.embedding
        t = m.table
        # ---- forward ----
        call("rs_embedding_lookup_fwd", s, ptr(self.ids), None, B, F, ptr(emb.row_base),
             ptr(emb.bucket), emb.hash_mode, emb.combiner, ptr(t.weight), t.rows, E, ptr(self.x0),
             F * E, E, ptr(self.rows))
        drop = il.dropout_rate if il.use_dropout else 0.0
        call("rs_il_fwd", s, ptr(self.x0), B, F, E, U, H, L, ptr(il.kernel), ptr(il.bias),
             ptr(il.gamma), ptr(il.beta), il.epsilon, int(il.use_res), drop, il.seed,
             self.cat.data_ptr() + 4 * D, CW, ptr(self.xsave) if L > 1 else None)
        x, ldx = self.x0, F * E
        deep_io = []
        for i, layer in enumerate(self.deep_layers):
            last = i == len(self.deep_layers) - 1
            y, ldy = (self.cat, CW) if last else (self.h[i], layer.units)
            call("rs_dense_fwd", s, ptr(x), B, layer.input_dim, ldx, ptr(layer.kernel), ptr(layer.bias),
                 layer.units, layer.act, ptr(y), ldy)
            deep_io.append((x, ldx, y, ldy))
            x, ldx = y, ldy
        x, ldx = self.cat, CW
        logit_io = []
        for j, layer in enumerate(self.logit_layers):
            last = j == len(self.logit_layers) - 1
            y, ldy = (self.s, self.T) if last else (self.lh[j], layer.units)
            call("rs_dense_fwd", s, ptr(x), B, layer.input_dim, ldx, ptr(layer.kernel), ptr(layer.bias),
                 layer.units, layer.act, ptr(y), ldy)
            logit_io.append((x, ldx, y, ldy))
            x, ldx = y, ldy
        call("rs_bce_clip_loss", s, ptr(self.s), ptr(self.labels), B, self.T, 1e-6, 1.0, 1e-6, None,
             ptr(self.p), ptr(self.loss), ptr(self.ds))
        # ---- backward ----
        dy, lddy = self.ds, self.T
        for j in reversed(range(len(self.logit_layers))):
            layer = self.logit_layers[j]
            x, ldx, y, ldy = logit_io[j]
            dx, lddx = (self.dcat, CW) if j == 0 else (self.dlh[j - 1], self.logit_layers[j - 1].units)
            call("rs_dense_bwd_data", s, ptr(dy), lddy, ptr(y), ldy, layer.act, ptr(layer.kernel), B,
                 layer.input_dim, layer.units, ptr(dx), lddx, 0)
            call("rs_dense_bwd_weight", s, ptr(x), ldx, ptr(dy), lddy, ptr(y), ldy, layer.act, B,
                 layer.input_dim, layer.units, self._grad(layer.kernel), self._grad(layer.bias), 0,
                 ptr(self.dense_ws), self.dense_ws_n)
            dy, lddy = dx, lddx
        dy_ptr, lddy = self.dcat.data_ptr(), CW   # deep part = dcat[:, :D]
        for i in reversed(range(len(self.deep_layers))):
            layer = self.deep_layers[i]
            x, ldx, y, ldy = deep_io[i]
            dx, lddx = (self.dx0, F * E) if i == 0 else (self.dh[i - 1], self.deep_layers[i - 1].units)
            call("rs_dense_bwd_data", s, dy_ptr, lddy, ptr(y), ldy, layer.act, ptr(layer.kernel), B,
                 layer.input_dim, layer.units, ptr(dx), lddx, 0)
            call("rs_dense_bwd_weight", s, ptr(x), ldx, dy_ptr, lddy, ptr(y), ldy, layer.act, B,
                 layer.input_dim, layer.units, self._grad(layer.kernel), self._grad(layer.bias), 0,
                 ptr(self.dense_ws), self.dense_ws_n)
            dy_ptr, lddy = ptr(dx), lddx
        call("rs_il_bwd", s, ptr(self.x0), ptr(self.xsave) if L > 1 else None,
             self.dcat.data_ptr() + 4 * D, CW, B, F, E, U, H, L, ptr(il.kernel), ptr(il.bias),
             ptr(il.gamma), ptr(il.beta), il.epsilon, int(il.use_res), drop, il.seed, ptr(self.dx0),
             1, ptr(self.il_dparams), 0, ptr(self.il_ws), self.il_ws_n)
        t.accumulate(self.rows, None, B, F, self.dx0, F * E, E, emb.combiner)

    def _exchange(self):
        """Data-parallel gradient exchange (recommendsystem_amd/dist.py)."""
        from .dist import allreduce_flat, exchange_packed, exchange_packed_merged, gather_sparse_lists
        m, t = self.model, self.model.table
        if self.packed_dp:
            if self.dp_sync_free:
                exchange_packed_merged(self.dp_buf, self.dp_all, self.pg)
                return
            self.dp_nmax = exchange_packed(self.dp_send, self.dp_recv, self.dp_n, self.dp_recs,
                                           self.dp_recs_all, self.dp_rs, self.pg)
            if self.dp_nmax > self.dp_cap:
                raise RuntimeError(f"sparse exchange: {self.dp_nmax} records > capacity {self.dp_cap}")
            return
        allreduce_flat(m.arena.grad, self.pg)
        scan = t.mode == "scan"
        if scan:
            call("rs_sparse_compact_scan", stream_handle(), ptr(t.grad), ptr(t.flag), t.rows, t.dim,
                 ptr(self.x_rows), ptr(self.x_grads), ptr(self.x_count), t.touched_cap)
            cnt = self.x_count
        else:
            cnt = t.n_touched[:1].clone()
            call("rs_sparse_compact", stream_handle(), ptr(t.grad), ptr(t.flag), ptr(t.touched),
                 ptr(t.n_touched), t.dim, ptr(self.x_rows), ptr(self.x_grads), t.touched_cap)
            t.n_touched[:1].zero_()  # (the sticky overflow word stays for check_overflow)
        rows_all, grads_all, n = gather_sparse_lists(self.x_rows, self.x_grads, cnt, self.pg)
        for r in range(self.world if n else 0):  # rank order -> identical sums on every replica
            call("rs_sparse_merge_rows", stream_handle(), ptr(rows_all[r]), ptr(grads_all[r]), n,
                 t.dim, ptr(t.grad), ptr(t.flag), None if scan else ptr(t.touched),
                 None if scan else ptr(t.n_touched), t.touched_cap)

    def dp_gathered_counts(self) -> torch.Tensor:
        """Every rank's record count of the last packed exchange, read from the gathered
        buffers (tests / diagnostics: the sync-free step itself never reads them on the host)."""
        if self.dp_sync_free:
            return self.dp_all.view(torch.int32).view(self.world, self.dp_S)[:, self.dp_n]
        return self.dp_recv.view(torch.int32).view(self.world, self.dp_ld)[:, self.dp_n]

    def _optimize(self):
        m, cfg = self.model, self.model.cfg
        ar = m.arena
        if self.head is not None and not self.dp:
            # partials -> grads -> Adam, one launch; a scan-mode table's sparse Adam runs in the
            # same launch on blocks of its own
            tail = self._scan_tail(m.table)
            # small batches: the sparse Adam walks the step's B x F looked-up rows (the only rows
            # its push marked) instead of sweeping the 2.6 M flags (rs_partials_reduce_adam_rows);
            # RS_SPARSE_ROWS_MAXN sets the largest B x F that does
            import os
            rows_max = int(os.environ.get("RS_SPARSE_ROWS_MAXN", str(ROWS_MODE_MAXN)))
            rows = (self.rows, self.B * self.F) if (tail is not None and
                                                    self.B * self.F <= rows_max) else None
            self._reduce_dense(adam=True, scan_table=tail, scan_rows=rows)
            if tail is None:
                m.table.step(grad_scale=1.0)
            return
        scale = 1.0 / self.world
        if self.packed_dp:
            s, t = stream_handle(), m.table
            if self.dp_sync_free:  # the merged layout: rank r's block at r * S
                gat, row_ld = self.dp_all, self.dp_S
                recs, stride = self.dp_all.data_ptr() + 4 * self.dp_ld, self.dp_S // self.dp_rs
            else:
                gat, row_ld = self.dp_recv, self.dp_ld
                recs, stride = self.dp_recs_all.data_ptr(), 0
            counts = gat.data_ptr() + 4 * self.dp_n
            for r in range(self.world):  # rank order: identical sums on every replica
                call("rs_sparse_merge_packed_stride", s, recs, counts, row_ld, self.world, r,
                     t.dim, ptr(t.grad), ptr(t.flag), t.rows, self.dp_cap, stride)
            # dense: rank-ordered sum of the gathered buckets -> arena grad -> Adam, one launch
            tail = self._scan_tail(t)
            # small per-rank batches: walk the gathered records (the rows the merges marked, at
            # most world x B_local x F) instead of sweeping the flags (rows mode, as at world 1)
            import os
            rows_max = int(os.environ.get("RS_SPARSE_ROWS_MAXN", str(ROWS_MODE_MAXN)))
            rows = None
            if tail is not None and self.dp_sync_free and self.B * self.F <= rows_max:
                # segment r = rank r's block seen as records from its record start: its first
                # count entries are rank r's records (the rest: padding / the next dense part)
                rows = (recs, self.world * stride, self.dp_rs, counts, row_ld, stride)
            _lib.partials_reduce_adam(s, [(ptr(gat), row_ld, self.world, self.dp_n,
                                           ptr(ar.grad), 1.0, 0)], ar.data, self.adam_m,
                                      self.adam_v, self.step_count, self.head["done"],
                                      cfg.lr_dense, 0.9, 0.999, 1e-8, scale, True,
                                      scan_table=tail, scan_grad_scale=scale, scan_rows=rows)
            if tail is None:
                t.step(grad_scale=scale)
            return
        call("rs_dense_adam", stream_handle(), ptr(ar.data), ptr(ar.grad), ptr(self.adam_m),
             ptr(self.adam_v), ar.n, ptr(self.step_count), cfg.lr_dense, 0.9, 0.999, 1e-8, scale, 0)
        m.table.step(grad_scale=scale)

    def _step_eager(self):
        self._forward_backward()
        if self.dp:
            self._exchange()
        self._optimize()

    # ---------------------------------------------------------------------------------------
    def load_batch(self, ids: torch.Tensor, labels: torch.Tensor) -> None:
        self.ids.copy_(ids, non_blocking=True)
        self.labels.copy_(labels.reshape(self.B, self.T), non_blocking=True)

    def _state(self):
        """Every tensor a training step mutates (dense arena + Adam moments + step counter, the
        table with its optimizer slots, gradient rows, flags and counters, the loss)."""
        m, t = self.model, self.model.table
        out = [m.arena.data, m.arena.grad, self.adam_m, self.adam_v, self.step_count, self.loss,
               t.weight, t.grad, t.flag, t.n_touched, t.touched]
        out += [t.m, t.v] if hasattr(t, "m") else [t.g2sum]
        if self.head is not None:
            out.append(self.head["done"])
        if self.metrics is not None:  # warm-up steps leave the metric totals untouched
            out += [mt.state for mt in self.metrics]
        return out

    def _warmup(self, steps: int) -> None:
        """Run `steps` eager steps on a side stream (first-launch initialisation before a capture)
        and then restore the training state: warm-up leaves parameters, optimizer state and the
        table exactly as they were."""
        if steps <= 0:
            return
        saved = [t.clone() for t in self._state()]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(steps):
                self._step_eager()
        torch.cuda.current_stream().wait_stream(side)
        for t, s in zip(self._state(), saved):
            t.copy_(s)
        torch.cuda.synchronize()

    def _record(self):
        """Record the step over the CURRENT self.ids / self.labels: one graph for the whole step
        (N = 1, or N > 1 on RCCL: the all-gather inside it), or the forward/backward half only
        (N > 1 on gloo: the collectives stay eager and the optimizer half is recorded once by
        _record_opt)."""
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=capture_error_mode()):
            if self._one_graph:
                self._step_eager()
            else:
                self._forward_backward()
        return g

    def _record_opt(self):
        if getattr(self, "graph_opt", None) is None:
            self.graph_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_opt, capture_error_mode=capture_error_mode()):
                self._optimize()

    def capture(self, warmup: int = 2) -> None:
        """Capture the step over the trainer's own static ids / labels buffers (``step()``
        replays it).  ``warmup`` eager steps run first and are rolled back (see _warmup)."""
        self._warmup(max(warmup, 1) if self.dp else warmup)
        if self._one_graph:
            self.graph = self._record()
        else:
            self.graph_fb = self._record()
            self._record_opt()
            self.graph = True

    def capture_pool(self, batches, warmup: int = 2) -> None:
        """One graph per device-resident batch [(ids, labels), ...]: each graph's lookup and loss
        read that batch's own buffers, so replaying batch i needs no copy into a static input
        (what a double-buffered loader hands over).  ``step_pool(i)`` replays batch i.
        Data parallel (N > 1): one forward/backward graph per batch plus ONE optimizer graph
        (it does not depend on the batch), the exchange between them eager.

        Every graph object is kept for the trainer's lifetime (self.pool_graphs; a graph owns a
        private memory pool).  Round 1's version re-ran capture() per batch, which replaced
        graph_opt each time and dropped the earlier ones while the forward/backward graphs
        recorded beside them stayed in use; that configuration faulted on its first replay in a
        2-rank rehearsal and was replaced by a single graph.  tests/test_gpu_dp.py replays
        several pairs of this layout alternately.  The trainer's own static buffers and its
        step() graph are untouched: step(ids, labels) still copies into them."""
        self.pool_batches = []
        for ids, labels in batches:
            if ids.shape != (self.B, self.F) or ids.dtype != torch.int64 or not ids.is_contiguous():
                raise ValueError("pool ids must be contiguous int64 [B, F]")
            self.pool_batches.append((ids, labels.reshape(self.B, self.T).float().contiguous()))
        own = (self.ids, self.labels)
        # (DP: at least one eager step, so the communicator exists before a capture uses it)
        self._warmup(max(warmup, 1) if self.dp else warmup)
        self.pool_graphs = []
        try:
            for ids, labels in self.pool_batches:
                self.ids, self.labels = ids, labels
                self.pool_graphs.append(self._record())
        finally:
            self.ids, self.labels = own
        if not self._one_graph:
            self._record_opt()
        self._prime_graphs()

    def _prime_graphs(self) -> None:
        """Replay every captured graph once and roll the training state back.  A hipGraph's
        first launch after capture is slower than the following ones (the runtime finishes
        setting up and uploading its executable; measured per step with RS_BENCH_STEP_TRACE):
        done here, as part of capture, so no training step pays it.  RS_NO_GRAPH_PRIME=1
        skips it (A/B)."""
        import os
        if os.environ.get("RS_NO_GRAPH_PRIME"):
            return
        saved = [t.clone() for t in self._state()]
        for g in self.pool_graphs:
            g.replay()
        if not self._one_graph and self.graph_opt is not None:
            self.graph_opt.replay()
        torch.cuda.synchronize()
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        torch.cuda.synchronize()

    def step_pool(self, i: int) -> torch.Tensor:
        g = self.pool_graphs[i % len(self.pool_graphs)]
        g.replay()
        if not self._one_graph:
            _lib.trace_point("graph_fb")
            self._exchange()
            _lib.trace_point("exchange")
            self.graph_opt.replay()
            _lib.trace_point("graph_opt")
        return self.loss

    def step(self, ids: torch.Tensor | None = None, labels: torch.Tensor | None = None) -> torch.Tensor:
        if ids is not None:
            self.load_batch(ids, labels)
        if self.graph is None:
            self._step_eager()
        elif self._one_graph:
            self.graph.replay()
        else:
            self.graph_fb.replay()
            self._exchange()
            self.graph_opt.replay()
        return self.loss
