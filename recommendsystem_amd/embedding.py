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

import ctypes
import os
from dataclasses import dataclass
from typing import Sequence

import torch
from torch import nn

from . import _lib
from ._lib import call, ptr, stream_handle

# grouped single-hot pushes in Trainer steps (RS_PUSH_GROUP=0: one launch per lookup layer, A/B)
_PUSH_GROUP = os.environ.get("RS_PUSH_GROUP", "1") != "0"

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
                 seed: int = 0, max_touched: int | None = None, initial: torch.Tensor | None = None):
        if dim % 4 != 0:
            raise ValueError("embedding dim must be a multiple of 4 (16-byte rows)")
        device = torch.device(device or "cuda")
        self.rows, self.dim = int(rows), int(dim)
        self.optimizer = optimizer or SparseAdam()
        if initial is not None:  # explicit initial rows (a ShardedSparseTable shard)
            if tuple(initial.shape) != (self.rows, self.dim):
                raise ValueError("initial must be [rows, dim]")
            w = initial
        else:
            w = self.initial_weight(self.rows, self.dim, self.optimizer, init_scale, seed)
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
        # a single-GPU Trainer switches tables with prefer_scan to scan mode (trainer.py)
        self.prefer_scan = False
        # deterministic pushes (rs_sparse_grad_accumulate_sorted: sort + segmented sum, bitwise
        # reproducible) instead of the LDS-hash + float-atomic push; workspace grown on demand
        self.deterministic = False
        self._sorted_ws = None
        self._push_ws = None
        # grouped pushes (begin_push_group / end_push_group, Trainer steps): the single-hot
        # pushes of one backward, recorded and issued as ONE rs_sparse_grad_accumulate_group
        self._deferred = None
        self._group_ws = None
        # autograd anchor: lets the lookup's backward run (it returns no dense gradient)
        self.anchor = torch.zeros((), device=device, dtype=torch.float32, requires_grad=True)

    @staticmethod
    def initial_weight(rows, dim, optimizer, init_scale=0.05, seed=0) -> torch.Tensor:
        """The table's initial values on the host: U(-s, s) from a seeded generator (AdaGrad:
        tn.core.AdaGrad's initial_scale)."""
        return SparseTable.initial_shard(rows, dim, optimizer, init_scale, seed, 0, 1)

    @staticmethod
    def initial_shard(rows, dim, optimizer, init_scale=0.05, seed=0, rank=0, world=1,
                      chunk_rows=1 << 16) -> torch.Tensor:
        """Rows rank, rank + world, ... of ``initial_weight(rows, ...)``, drawn in row chunks from
        the same seeded stream (a chunked draw continues the generator exactly where one draw of
        the whole table would be), so a rank holds only its shard plus one chunk on the host."""
        gen = torch.Generator().manual_seed(seed)
        scale = init_scale
        if isinstance(optimizer, SparseAdaGrad):
            scale = optimizer.initial_scale / max(init_scale, 1e-30)
        parts = []
        for r0 in range(0, rows, chunk_rows):
            n = min(chunk_rows, rows - r0)
            w = (torch.rand(n, dim, generator=gen) * 2.0 - 1.0) * init_scale
            if isinstance(optimizer, SparseAdaGrad):
                w = w * scale
            parts.append(w[(rank - r0) % world::world].clone() if world > 1 else w)
        return torch.cat(parts) if parts else torch.empty(0, dim)

    # ---- push / update -----------------------------------------------------------------
    def _groupable(self, offsets, dout, dout_ld, dout_fstride) -> bool:
        """rs_sparse_grad_accumulate_group's domain: single-hot, >= 32-float rows, 16-B aligned
        gradient rows, the non-deterministic push."""
        return (offsets is None and not self.deterministic and self.dim >= 32 and
                dout.data_ptr() % 16 == 0 and dout_ld % 4 == 0 and dout_fstride % 4 == 0)

    def begin_push_group(self) -> None:
        """Record this table's single-hot pushes until end_push_group (one backward's pushes
        from several lookup layers into this table: staytime/VideoDnn.py:217-244 declares every
        column of the shared table in ONE tn.layers.EmbeddingFeatures)."""
        if _PUSH_GROUP:
            self._deferred = []

    def end_push_group(self) -> None:
        """Issue the recorded pushes: one grouped launch (+ one claim launch) per <= 8 sources."""
        d, self._deferred = self._deferred, None
        if not d:
            return
        for k0 in range(0, len(d), 8):
            chunk = d[k0:k0 + 8]
            if len(chunk) == 1:
                rows, B, F, dout, ld, fs = chunk[0]
                self.accumulate(rows, None, B, F, dout, ld, fs, 0)
                continue
            n = len(chunk)
            keep = [_lib.c_array(ctypes.c_void_p, [ptr(c[0]) for c in chunk]),
                    _lib.c_array(ctypes.c_void_p, [ptr(c[3]) for c in chunk]),
                    _lib.c_array(ctypes.c_int64, [c[1] for c in chunk]),
                    _lib.c_array(ctypes.c_int32, [c[2] for c in chunk]),
                    _lib.c_array(ctypes.c_int64, [c[4] for c in chunk]),
                    _lib.c_array(ctypes.c_int64, [c[5] for c in chunk])]  # (alive for the calls)
            rp, dp, bp, fp, lp, sp = (a for _, a in keep)
            scan = self.mode == "scan"
            ws, wsn = None, 0
            if not scan:
                need = int(_lib.load().rs_sparse_push_group_workspace_bytes(n, bp, fp))
                if need < 0:
                    raise ValueError("grouped push: unsupported source shapes")
                if self._group_ws is None or self._group_ws.numel() < need:
                    self._group_ws = torch.empty(need, device=self.weight.device, dtype=torch.uint8)
                ws, wsn = ptr(self._group_ws), self._group_ws.numel()
            call("rs_sparse_grad_accumulate_group", stream_handle(), n, rp, dp, bp, fp, lp, sp,
                 self.dim, ptr(self.grad), ptr(self.flag), None if scan else ptr(self.touched),
                 None if scan else ptr(self.n_touched), self.touched_cap, ws, wsn)

    def accumulate(self, rows: torch.Tensor, offsets: torch.Tensor | None, B: int, F: int,
                   dout: torch.Tensor, dout_ld: int, dout_fstride: int, combiner: int) -> None:
        if self._deferred is not None and self._groupable(offsets, dout, dout_ld, dout_fstride):
            # (the record keeps rows / dout alive until the grouped launch reads them)
            self._deferred.append((rows, int(B), int(F), dout, int(dout_ld), int(dout_fstride)))
            return
        scan = self.mode == "scan"
        if self.deterministic:
            n = rows.numel()
            ws = self.sorted_workspace(n)
            call("rs_sparse_grad_accumulate_sorted", stream_handle(), ptr(rows), ptr(offsets), B, F,
                 ptr(dout), dout_ld, dout_fstride, self.dim, combiner, self.rows, ptr(self.grad),
                 ptr(self.flag), None if scan else ptr(self.touched),
                 None if scan else ptr(self.n_touched), self.touched_cap, ptr(ws), ws.numel(), n)
            return
        # single-hot list-mode pushes claim rows by election (csrc/embedding.hip rs_push): a
        # workspace of candidate rows per push block, kept and grown on demand (a captured graph
        # reuses the one its warm-up step allocated)
        ws, wsn = None, 0
        if offsets is None and not scan:
            need = int(_lib.load().rs_sparse_push_workspace_bytes(B, F))
            if self._push_ws is None or self._push_ws.numel() < need:
                self._push_ws = torch.empty(need, device=self.weight.device, dtype=torch.uint8)
            ws, wsn = ptr(self._push_ws), self._push_ws.numel()
        call("rs_sparse_grad_accumulate_ws", stream_handle(), ptr(rows), ptr(offsets), B, F,
             ptr(dout), dout_ld, dout_fstride, self.dim, combiner, ptr(self.grad), ptr(self.flag),
             None if scan else ptr(self.touched), None if scan else ptr(self.n_touched),
             self.touched_cap, ws, wsn)

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
        n_touched[288]; the rows past touched_cap are still updated, by the recovery sweep of
        ``step``, which runs every step until this check clears the word).  Reads the device:
        call it outside the timed / captured region."""
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
        # a touched list smaller than the table can overflow: the gated sweep after the list
        # launch updates the claimed rows it could not hold (exits at once otherwise)
        recover = self.touched_cap < self.rows
        if isinstance(o, SparseAdam):
            call("rs_sparse_adam", s, ptr(self.weight), ptr(self.m), ptr(self.v), ptr(self.grad),
                 ptr(self.flag), ptr(self.touched), ptr(self.n_touched), self.dim,
                 self.touched_cap, o.learning_rate, o.beta1, o.beta2, o.epsilon, grad_scale)
            if recover:
                call("rs_sparse_adam_recover", s, ptr(self.weight), ptr(self.m), ptr(self.v),
                     ptr(self.grad), ptr(self.flag), ptr(self.n_touched), self.rows, self.dim,
                     o.learning_rate, o.beta1, o.beta2, o.epsilon, grad_scale)
        else:
            call("rs_sparse_adagrad", s, ptr(self.weight), ptr(self.g2sum), ptr(self.grad),
                 ptr(self.flag), ptr(self.touched), ptr(self.n_touched), self.dim,
                 self.touched_cap, o.learning_rate, grad_scale)
            if recover:
                call("rs_sparse_adagrad_recover", s, ptr(self.weight), ptr(self.g2sum),
                     ptr(self.grad), ptr(self.flag), ptr(self.n_touched), self.rows, self.dim,
                     o.learning_rate, grad_scale)


class ShardedSparseTable:
    """N2 owner-sharded table: the rows of a SparseTable of ``rows`` rows split over
    the ``world`` ranks of a process group by owner = row % world; this rank keeps rows rank,
    rank + world, ... (local index row // world) with their optimizer slots, as ``local``, a
    SparseTable of ceil((rows - rank) / world) rows.  Initial values equal the replicated
    SparseTable(rows, seed=seed)'s rows.  Lookups hash ids to global rows on the requesting rank,
    route them to their owners (rs_owner_route + all_to_all_v), the owners gather
    (rs_gather_rows) and send the rows back (rs_scatter_rows into id order); backward sends the
    per-id gradients the same way and the owner pushes them into its shard, so the sparse
    optimizer step (``step``) is local and no table-sized exchange runs.

    Two routings.  ``owner_cap=None``: variable splits, the per-owner counts exchanged and read
    on the host once per lookup (exact sizes, one host synchronisation per lookup).
    ``owner_cap=c``: sync-free -- each (requester, owner) pair has a fixed block of c id slots
    (rs_owner_route_fixed), so every all-to-all has equal splits known in advance, nothing is read
    back and the whole step can be captured in one HIP graph (Trainer.capture_pool under RCCL);
    a lookup that sends more than c ids to one owner drops the excess and records it in the sticky
    ``route_stats`` word, which ``check_overflow`` reports (Trainer.measure_dp_caps sizes c from
    the batches).  Everything else (``weight``, ``grad``, ``optimizer``, ``step``, ...) is the
    local shard's."""

    sharded = True

    def __init__(self, rows: int, dim: int, optimizer=None, device=None, init_scale: float = 0.05,
                 seed: int = 0, max_touched: int | None = None, process_group=None,
                 owner_cap: int | None = None):
        import torch.distributed as dist
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.rows, self.dim = int(rows), int(dim)
        if self.rows > 2**31 - 1:
            raise ValueError("row indices are int32")
        optimizer = optimizer or SparseAdam()
        shard = SparseTable.initial_shard(self.rows, self.dim, optimizer, init_scale, seed,
                                          self.rank, self.world)
        self.local = SparseTable(shard.shape[0], dim, optimizer, device=device, initial=shard,
                                 max_touched=max_touched)
        self._route_ws = None
        self.owner_cap = None if owner_cap is None else int(owner_cap)
        # [0]: the largest ids one lookup sent to one owner (sticky; device, fixed routing)
        self.route_stats = torch.zeros(1, device=self.local.weight.device, dtype=torch.int32)
        self.peak_owner_ids = 0  # the same on the host (variable routing: from the counts it reads)

    def __getattr__(self, name):  # the shard's state and methods
        if name == "local":
            raise AttributeError(name)
        return getattr(self.local, name)

    @property
    def deterministic(self):
        return self.local.deterministic

    @deterministic.setter
    def deterministic(self, v):
        self.local.deterministic = bool(v)

    @property
    def mode(self):
        return self.local.mode

    @mode.setter
    def mode(self, v):
        self.local.mode = v

    def _workspace(self, n):
        need = int(_lib.load().rs_owner_route_workspace_bytes(n, self.world))
        if need < 0:
            raise ValueError(f"{n} ids / world {self.world}: out of range for the owner route")
        if self._route_ws is None or self._route_ws.numel() < need:
            self._route_ws = torch.empty(need, device=self.local.weight.device, dtype=torch.uint8)
        return self._route_ws

    def check_overflow(self) -> None:
        """The shard's touched-list check, and (fixed routing) whether a lookup sent more ids to
        one owner than owner_cap (those ids were dropped).  Reads the device."""
        self.local.check_overflow()
        if self.owner_cap is not None:
            n = int(self.route_stats[0].item())
            if n > self.owner_cap:
                self.route_stats.zero_()
                raise RuntimeError(f"sharded table routing overflow: a lookup sent {n} ids to one "
                                   f"owner, owner_cap is {self.owner_cap} (raise owner_cap)")

    def route(self, rows: torch.Tensor):
        """Global rows int32 [n] (-1 = no row) -> the routing plan shared by gather and push.
        Variable routing: ("v", send_pos [nv], send_splits, recv_splits, recv_local [nr]);
        fixed routing: ("f", slot [n], recv_local [world * owner_cap])."""
        if self.owner_cap is not None:
            return self._route_fixed(rows)
        from .dist import all_to_all_v, exchange_counts
        n, dev = rows.numel(), rows.device
        send_local = torch.empty(n, device=dev, dtype=torch.int32)
        send_pos = torch.empty(n, device=dev, dtype=torch.int32)
        counts = torch.empty(self.world, device=dev, dtype=torch.int32)
        ws = self._workspace(n)
        call("rs_owner_route", stream_handle(), ptr(rows), n, self.world, self.rows, ptr(send_local),
             ptr(send_pos), ptr(counts), ptr(ws), ws.numel())
        sc, rc = exchange_counts(counts, self.pg)
        self.peak_owner_ids = max(self.peak_owner_ids, max(sc, default=0))
        nv, nr = sum(sc), sum(rc)
        recv_local = torch.empty(nr, device=dev, dtype=torch.int32)
        all_to_all_v(recv_local, send_local[:nv], rc, sc, self.pg)
        return "v", send_pos[:nv], sc, rc, recv_local

    def _route_fixed(self, rows: torch.Tensor):
        from .dist import all_to_all_fixed
        n, dev, c = rows.numel(), rows.device, self.owner_cap
        send_local = torch.empty(self.world * c, device=dev, dtype=torch.int32)
        slot = torch.empty(n, device=dev, dtype=torch.int32)
        ws = self._workspace(n)
        call("rs_owner_route_fixed", stream_handle(), ptr(rows), n, self.world, self.rows, c,
             ptr(send_local), ptr(slot), ptr(self.route_stats), ptr(ws), ws.numel())
        recv_local = torch.empty_like(send_local)
        all_to_all_fixed(recv_local, send_local, self.pg)
        return "f", slot, recv_local

    def gather(self, rows: torch.Tensor):
        """-> (E [n, dim] with E[k] = table[rows[k]] (zero where rows[k] < 0), plan)."""
        from .dist import all_to_all_fixed, all_to_all_v
        plan = self.route(rows)
        dev, d = rows.device, self.dim
        if plan[0] == "f":  # fixed blocks: pads (-1) gather zero rows, slot -1 reads a zero row
            _, slot, recv_local = plan
            served = torch.empty(recv_local.numel(), d, device=dev)
            call("rs_gather_rows", stream_handle(), ptr(self.local.weight), d, ptr(recv_local),
                 recv_local.numel(), d, ptr(served), d)
            back = torch.empty_like(served)
            all_to_all_fixed(back, served, self.pg)
            E = torch.empty(rows.numel(), d, device=dev)
            if rows.numel():
                call("rs_gather_rows", stream_handle(), ptr(back), d, ptr(slot), rows.numel(), d,
                     ptr(E), d)
            return E, plan
        _, send_pos, sc, rc, recv_local = plan
        served = torch.empty(recv_local.numel(), d, device=dev)
        if served.numel():
            call("rs_gather_rows", stream_handle(), ptr(self.local.weight), d, ptr(recv_local),
                 recv_local.numel(), d, ptr(served), d)
        back = torch.empty(send_pos.numel(), d, device=dev)
        all_to_all_v(back, served, sc, rc, self.pg)
        E = torch.zeros(rows.numel(), d, device=dev)
        if back.numel():
            call("rs_scatter_rows", stream_handle(), ptr(back), d, ptr(send_pos), send_pos.numel(),
                 d, ptr(E), d)
        return E, plan

    def push(self, dE: torch.Tensor, plan) -> None:
        """Per-id gradients dE [n, dim] (the rows of gather's E) -> the owners' gradient rows."""
        from .dist import all_to_all_fixed, all_to_all_v
        d = self.dim
        if plan[0] == "f":  # pad slots travel unwritten: their row at the owner is -1 (skipped)
            _, slot, recv_local = plan
            g = torch.empty(recv_local.numel(), d, device=dE.device)
            if slot.numel():
                call("rs_scatter_rows", stream_handle(), ptr(dE), d, ptr(slot), slot.numel(), d,
                     ptr(g), d)
            recv = torch.empty_like(g)
            all_to_all_fixed(recv, g, self.pg)
            self.local.accumulate(recv_local, None, recv_local.numel(), 1, recv, d, d,
                                  COMBINERS["sum"])
            return
        _, send_pos, sc, rc, recv_local = plan
        g = torch.empty(send_pos.numel(), d, device=dE.device)
        if g.numel():
            call("rs_gather_rows", stream_handle(), ptr(dE), d, ptr(send_pos), send_pos.numel(), d,
                 ptr(g), d)
        recv = torch.empty(recv_local.numel(), d, device=dE.device)
        all_to_all_v(recv, g, rc, sc, self.pg)
        if recv.numel():
            self.local.accumulate(recv_local, None, recv_local.numel(), 1, recv, d, d,
                                  COMBINERS["sum"])


def is_sharded(table) -> bool:
    return getattr(type(table), "sharded", False)


class _ShardedLookupFn(torch.autograd.Function):
    """EmbeddingFeatures over a ShardedSparseTable: rows-only hash, remote gather, local pooling
    (VarLen: rs_embedding_lookup_fwd over the gathered per-id rows as a table indexed by id
    position); backward expands the combiner (rs_segment_expand) and pushes to the owners."""

    @staticmethod
    def forward(ctx, anchor, ids, offsets, layer, out_buf):
        B, F = layer._batch_fields(ids, offsets)
        t = layer.table
        n, d, dev, s = ids.numel(), t.dim, ids.device, stream_handle()
        rows = torch.empty(n, device=dev, dtype=torch.int32)
        call("rs_embedding_lookup_fwd", s, ptr(ids), ptr(offsets), B, F, ptr(layer.row_base),
             ptr(layer.bucket), layer.hash_mode, layer.combiner, None, t.rows, d, None, F * d, d,
             ptr(rows))
        E, plan = t.gather(rows)
        out = out_buf if out_buf is not None else torch.empty(B, F, d, device=dev)
        if offsets is None:
            out.view(B * F, d).copy_(E)
        elif n == 0:
            out.zero_()
        else:
            pos = torch.arange(n, device=dev, dtype=torch.int64)
            base = torch.zeros(F, device=dev, dtype=torch.int64)
            bucket = torch.full((F,), n, device=dev, dtype=torch.int64)
            call("rs_embedding_lookup_fwd", s, ptr(pos), ptr(offsets), B, F, ptr(base), ptr(bucket),
                 HASH_MODES["mod"], layer.combiner, ptr(E), n, d, ptr(out), F * d, d, None)
        ctx.layer, ctx.B, ctx.F, ctx.n, ctx.plan = layer, B, F, n, plan
        ctx.save_for_backward(offsets if offsets is not None else torch.empty(0))
        ctx.has_offsets = offsets is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        (offsets,) = ctx.saved_tensors
        layer, d = ctx.layer, ctx.layer.table.dim
        dout = dout.contiguous()
        if not ctx.has_offsets:
            dE = dout.view(ctx.B * ctx.F, d)  # one id per segment: every combiner scales by 1
        else:
            dE = torch.empty(ctx.n, d, device=dout.device)
            call("rs_segment_expand", stream_handle(), ptr(dout), ctx.F * d, d, ptr(offsets), ctx.B,
                 ctx.F, layer.combiner, d, ptr(dE))
        layer.table.push(dE, ctx.plan)
        return None, None, None, None, None


class _ShardedSeqLookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, offsets, layer):
        t = layer.table
        B, T, d, dev = offsets.numel() - 1, layer.seq_max_len, t.dim, ids.device
        mask = torch.empty(B, T, device=dev, dtype=torch.uint8)
        lengths = torch.empty(B, device=dev, dtype=torch.int32)
        rows = torch.empty(B * T, device=dev, dtype=torch.int32)
        call("rs_sequence_lookup_fwd", stream_handle(), ptr(ids), ptr(offsets), B, T,
             layer.row_base, layer.bucket, layer.hash_mode, None, d, None, T * d, d, ptr(mask), T,
             ptr(lengths), ptr(rows))
        E, plan = t.gather(rows)
        ctx.layer, ctx.B, ctx.plan = layer, B, plan
        ctx.mark_non_differentiable(mask, lengths)
        ctx.set_materialize_grads(False)  # no zero-filled grads for mask / lengths
        return E.view(B, T, d), mask.view(torch.bool), lengths

    @staticmethod
    def backward(ctx, dout, _dmask, _dlen):
        if dout is None:
            return None, None, None, None
        d = ctx.layer.table.dim
        ctx.layer.table.push(dout.contiguous().view(-1, d), ctx.plan)
        return None, None, None, None


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
        fn = _ShardedLookupFn if is_sharded(self.table) else _LookupFn
        return fn.apply(self.table.anchor, ids, offsets, self, out)


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
        ctx.set_materialize_grads(False)  # no zero-filled grads for mask / lengths
        return out, mask.view(torch.bool), lengths

    @staticmethod
    def backward(ctx, dout, _dmask, _dlen):
        if dout is None:
            return None, None, None, None
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
        fn = _ShardedSeqLookupFn if is_sharded(self.table) else _SeqLookupFn
        emb, mask, lengths = fn.apply(self.table.anchor, ids.reshape(-1).contiguous(), offsets, self)
        return (emb, mask, lengths) if return_lengths else (emb, mask)
