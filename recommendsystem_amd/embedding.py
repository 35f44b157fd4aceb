"""Sparse embedding front end: the tensornet boundary of the path.

    SparseTable         the PS-side table of tn.layers.EmbeddingFeatures + its sparse optimizer
                        state, resident in HBM (a 10M x 32 fp32 table is 1.28 GB of 288 GB)
    SparseAdam /        tn.core.Adam / tn.core.AdaGrad handed to EmbeddingFeatures
    SparseAdaGrad       (rank/ctr/base_model.py:163, rank/multi_head/multidnn.py:235,
                        staytime/VideoDnn.py:233)
    EmbeddingFeatures   tn.layers.EmbeddingFeatures(embedding_columns, sparse_opt)(inputs) for a
                        group of category columns sharing one table (per-field row ranges),
                        combiner 'mean' | 'sum' | 'sqrtn' (embedding_column), output [B, F, dim]
                        = the expand + Concatenate(axis=1) of autoint:22-26 already applied.

id -> row (tensornet's hash map is not vendored; pinned, identical in oracle/ctr_oracle.py):
    row = row_base[f] + H(id) mod bucket[f],  H = identity ('mod') or splitmix64 ('splitmix').
Backward pushes the pooled-output gradient into the table's gradient rows (fp32 atomics, rows
claimed once per step); ``SparseAdam.step`` updates exactly the touched rows.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle

HASH_MODES = {"mod": 0, "splitmix": 1}
COMBINERS = {"sum": 0, "mean": 1, "sqrtn": 2}


@dataclass
class SparseAdam:
    """tn.core.Adam(learning_rate, beta1, beta2, epsilon) as a sparse (per-row) optimizer.
    Form pinned to tensornet's SparseAdamValue (no bias correction); see csrc/optim.hip."""
    learning_rate: float = 5e-5
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8

    def slots(self) -> int:
        return 2


@dataclass
class SparseAdaGrad:
    """tn.core.AdaGrad(learning_rate, initial_g2sum, initial_scale) (staytime/VideoDnn.py:233)."""
    learning_rate: float = 0.005
    initial_g2sum: float = 0.1
    initial_scale: float = 0.1

    def slots(self) -> int:
        return 1


class SparseTable:
    """One HBM-resident embedding table with its optimizer slots and step bookkeeping."""

    def __init__(self, rows: int, dim: int, optimizer=None, device=None, init_scale: float = 0.05,
                 seed: int = 0, max_touched: int | None = None):
        if dim % 4 != 0:
            raise ValueError("embedding dim must be a multiple of 4 (16-byte rows)")
        device = torch.device(device or "cuda")
        self.rows, self.dim = int(rows), int(dim)
        self.optimizer = optimizer or SparseAdam()
        gen = torch.Generator().manual_seed(seed)
        w = (torch.rand(self.rows, self.dim, generator=gen) * 2.0 - 1.0) * init_scale
        if isinstance(self.optimizer, SparseAdaGrad):
            w = w * (self.optimizer.initial_scale / max(init_scale, 1e-30))
        self.weight = w.to(device=device, dtype=torch.float32)
        self.grad = torch.zeros(self.rows, self.dim, device=device, dtype=torch.float32)
        self.flag = torch.full((self.rows,), -1, device=device, dtype=torch.int32)
        cap = int(min(self.rows, max_touched)) if max_touched else self.rows
        self.touched_cap = cap
        self.touched = torch.zeros(cap, device=device, dtype=torch.int32)
        # {count, completion counters (csrc/common.hpp RS_DONE_WORDS), overflow word}
        self.n_touched = torch.zeros(1 + 288, device=device, dtype=torch.int32)
        if isinstance(self.optimizer, SparseAdam):
            self.m = torch.zeros_like(self.weight)
            self.v = torch.zeros_like(self.weight)
        else:
            self.g2sum = torch.full_like(self.weight, self.optimizer.initial_g2sum)
        # "list": pushes claim rows into `touched` (grid sized by touched_cap); "scan": pushes only
        # mark flag[] and the optimizer sweeps it (no returning atomics in the push; best when
        # the table is not much larger than ~100x the rows a step touches)
        self.mode = "list"
        # deterministic pushes (rs_sparse_grad_accumulate_sorted: sort + segmented sum, bitwise
        # reproducible) instead of the LDS-hash + float-atomic push; workspace grown on demand
        self.deterministic = False
        self._sorted_ws = None
        # autograd anchor: lets the lookup's backward run (it returns no dense gradient)
        self.anchor = torch.zeros((), device=device, dtype=torch.float32, requires_grad=True)

    # ---- push / update -----------------------------------------------------------------
    def accumulate(self, rows: torch.Tensor, offsets: torch.Tensor | None, B: int, F: int,
                   dout: torch.Tensor, dout_ld: int, dout_fstride: int, combiner: int) -> None:
        scan = self.mode == "scan"
        if self.deterministic:
            n = rows.numel()
            ws = self.sorted_workspace(n)
            call("rs_sparse_grad_accumulate_sorted", stream_handle(), ptr(rows), ptr(offsets), B, F,
                 ptr(dout), dout_ld, dout_fstride, self.dim, combiner, self.rows, ptr(self.grad),
                 ptr(self.flag), None if scan else ptr(self.touched),
                 None if scan else ptr(self.n_touched), self.touched_cap, ptr(ws), ws.numel(), n)
            return
        call("rs_sparse_grad_accumulate", stream_handle(), ptr(rows), ptr(offsets), B, F, ptr(dout),
             dout_ld, dout_fstride, self.dim, combiner, ptr(self.grad), ptr(self.flag),
             None if scan else ptr(self.touched), None if scan else ptr(self.n_touched),
             self.touched_cap)

    def sorted_workspace(self, n_ids: int) -> torch.Tensor:
        """Workspace of the deterministic push for n_ids ids (kept and reused; reserve the
        largest batch before capturing a graph)."""
        need = int(_lib.load().rs_sparse_sorted_workspace_bytes(n_ids))
        if need < 0:
            raise ValueError(f"{n_ids} ids: too many for the deterministic push")
        if self._sorted_ws is None or self._sorted_ws.numel() < need:
            self._sorted_ws = torch.empty(need, device=self.weight.device, dtype=torch.uint8)
        return self._sorted_ws

    def check_overflow(self) -> None:
        """Raise if any step since the last check claimed more rows than the touched list holds
        (list mode; csrc/optim.hip records the largest such count in the sticky word
        n_touched[288] and updates only the first touched_cap rows).  Reads the device: call it
        outside the timed / captured region."""
        n = int(self.n_touched[288].item())
        if n:
            self.n_touched[288].zero_()
            raise RuntimeError(f"sparse table touched-row overflow: a step claimed {n} rows, the "
                               f"touched list holds {self.touched_cap} (raise max_touched)")

    def step(self, grad_scale: float = 1.0) -> None:
        """Apply the sparse optimizer to the rows touched since the last step."""
        o = self.optimizer
        s = stream_handle()
        if self.mode == "scan":
            if isinstance(o, SparseAdam):
                call("rs_sparse_adam_scan", s, ptr(self.weight), ptr(self.m), ptr(self.v),
                     ptr(self.grad), ptr(self.flag), self.rows, self.dim, o.learning_rate, o.beta1,
                     o.beta2, o.epsilon, grad_scale)
            else:
                call("rs_sparse_adagrad_scan", s, ptr(self.weight), ptr(self.g2sum), ptr(self.grad),
                     ptr(self.flag), self.rows, self.dim, o.learning_rate, grad_scale)
            return
        if isinstance(o, SparseAdam):
            call("rs_sparse_adam", s, ptr(self.weight), ptr(self.m), ptr(self.v), ptr(self.grad),
                 ptr(self.flag), ptr(self.touched), ptr(self.n_touched), self.dim,
                 self.touched_cap, o.learning_rate, o.beta1, o.beta2, o.epsilon, grad_scale)
        else:
            call("rs_sparse_adagrad", s, ptr(self.weight), ptr(self.g2sum), ptr(self.grad),
                 ptr(self.flag), ptr(self.touched), ptr(self.n_touched), self.dim,
                 self.touched_cap, o.learning_rate, grad_scale)


class _LookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, offsets, layer, out_buf):
        B, F = layer._batch_fields(ids, offsets)
        t = layer.table
        out = out_buf if out_buf is not None else torch.empty(
            B, F, t.dim, device=ids.device, dtype=torch.float32)
        rows = torch.empty(ids.numel(), device=ids.device, dtype=torch.int32)
        call("rs_embedding_lookup_fwd", stream_handle(), ptr(ids), ptr(offsets), B, F,
             ptr(layer.row_base), ptr(layer.bucket), layer.hash_mode, layer.combiner, ptr(t.weight),
             t.rows, t.dim, ptr(out), F * t.dim, t.dim, ptr(rows))
        ctx.layer, ctx.B, ctx.F = layer, B, F
        ctx.save_for_backward(rows, offsets if offsets is not None else torch.empty(0))
        ctx.has_offsets = offsets is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        rows, offsets = ctx.saved_tensors
        layer = ctx.layer
        dout = dout.contiguous()
        layer.table.accumulate(rows, offsets if ctx.has_offsets else None, ctx.B, ctx.F, dout,
                               ctx.F * layer.table.dim, layer.table.dim, layer.combiner)
        return None, None, None, None, None


class EmbeddingFeatures(nn.Module):
    """tn.layers.EmbeddingFeatures over F category columns that share one SparseTable.

    ``buckets[f]`` is category_column(key, bucket_size).bucket_size of field f; fields get
    disjoint row ranges [row_base[f], row_base[f] + buckets[f]) unless ``row_base`` is given
    (equal bases = one shared hashed space, e.g. the 10M-row table of config 5).
    Input: ids int64 [B, F] (one id per field) or (ids [nnz], offsets int32 [B*F + 1]) for
    variable-length (VarLen) features.  Output: [B, F, dim].
    """

    def __init__(self, table: SparseTable, buckets: Sequence[int], row_base: Sequence[int] | None = None,
                 combiner: str = "mean", hash_mode: str = "mod"):
        super().__init__()
        self.table = table
        F = len(buckets)
        if row_base is None:
            row_base, acc = [], 0
            for bk in buckets:
                row_base.append(acc)
                acc += int(bk)
        if len(row_base) != F:
            raise ValueError("row_base and buckets must have one entry per field")
        for rb, bk in zip(row_base, buckets):
            if rb < 0 or bk <= 0 or rb + bk > table.rows:
                raise ValueError(f"field rows [{rb}, {rb + bk}) outside the table ({table.rows} rows)")
        dev = table.weight.device
        self.num_fields = F
        self.row_base = torch.tensor([int(r) for r in row_base], dtype=torch.int64, device=dev)
        self.bucket = torch.tensor([int(b) for b in buckets], dtype=torch.int64, device=dev)
        self.combiner = COMBINERS[combiner]
        self.hash_mode = HASH_MODES[hash_mode]

    def _batch_fields(self, ids, offsets):
        F = self.num_fields
        if offsets is None:
            if ids.dim() != 2 or ids.shape[1] != F:
                raise ValueError(f"ids must be [B, {F}] int64 when no offsets are given")
            return ids.shape[0], F
        if (offsets.numel() - 1) % F != 0:
            raise ValueError("offsets must have B*F + 1 entries")
        return (offsets.numel() - 1) // F, F

    def forward(self, ids: torch.Tensor, offsets: torch.Tensor | None = None, out: torch.Tensor | None = None):
        _lib.require_device(ids)
        if ids.dtype != torch.int64:
            raise TypeError("ids must be int64 (tn.layers.Input(dtype='int64'))")
        ids = ids.contiguous()
        if offsets is not None:
            offsets = offsets.to(torch.int32).contiguous()
        return _LookupFn.apply(self.table.anchor, ids, offsets, self, out)


class _SeqLookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, offsets, layer):
        t = layer.table
        B, T = offsets.numel() - 1, layer.seq_max_len
        dev = ids.device
        out = torch.empty(B, T, t.dim, device=dev, dtype=torch.float32)
        mask = torch.empty(B, T, device=dev, dtype=torch.uint8)
        lengths = torch.empty(B, device=dev, dtype=torch.int32)
        rows = torch.empty(B * T, device=dev, dtype=torch.int32)
        call("rs_sequence_lookup_fwd", stream_handle(), ptr(ids), ptr(offsets), B, T,
             layer.row_base, layer.bucket, layer.hash_mode, ptr(t.weight), t.dim, ptr(out), T * t.dim,
             t.dim, ptr(mask), T, ptr(lengths), ptr(rows))
        ctx.layer, ctx.B = layer, B
        ctx.save_for_backward(rows)
        ctx.mark_non_differentiable(mask, lengths)
        return out, mask.view(torch.bool), lengths

    @staticmethod
    def backward(ctx, dout, _dmask, _dlen):
        (rows,) = ctx.saved_tensors
        layer = ctx.layer
        T, dim = layer.seq_max_len, layer.table.dim
        layer.table.accumulate(rows, None, ctx.B, T, dout.contiguous(), T * dim, dim, COMBINERS["sum"])
        return None, None, None, None


class SequenceEmbedding(nn.Module):
    """embedding_column(categorical_column, dimension, combiner=None, seq_max_len) of
    tn.layers.EmbeddingFeatures (staytime/VideoDnn.py:217-244): a VarLen id list per sample ->
    (emb [B, seq_max_len, dim], mask [B, seq_max_len] bool).  Pinned: the first seq_max_len ids
    are kept; padding rows are zero and receive no gradient.  Input: ids int64 [nnz] +
    offsets int32 [B + 1], or a dense [B, n] id matrix (every row full)."""

    def __init__(self, table: SparseTable, bucket: int, seq_max_len: int, row_base: int = 0,
                 hash_mode: str = "mod"):
        super().__init__()
        if row_base < 0 or bucket <= 0 or row_base + bucket > table.rows:
            raise ValueError(f"rows [{row_base}, {row_base + bucket}) outside the table")
        self.table = table
        self.bucket, self.row_base = int(bucket), int(row_base)
        self.seq_max_len = int(seq_max_len)
        self.hash_mode = HASH_MODES[hash_mode]

    def forward(self, ids: torch.Tensor, offsets: torch.Tensor | None = None,
                return_lengths: bool = False):
        """-> (emb, mask) like tensornet, or (emb, mask, lengths int32 [B]) with return_lengths."""
        _lib.require_device(ids)
        if ids.dtype != torch.int64:
            raise TypeError("ids must be int64")
        if offsets is None:
            if ids.dim() != 2:
                raise ValueError("ids must be [B, n] when no offsets are given")
            B, n = ids.shape
            offsets = torch.arange(0, B * n + 1, n, device=ids.device, dtype=torch.int32)
        offsets = offsets.to(device=ids.device, dtype=torch.int32).contiguous()
        emb, mask, lengths = _SeqLookupFn.apply(self.table.anchor, ids.reshape(-1).contiguous(), offsets, self)
        return (emb, mask, lengths) if return_lengths else (emb, mask)
