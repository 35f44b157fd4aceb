"""Generic training step for the composed models (rank/multi_head, rough_rank, staytime, DIN
harness): what tensornet's ``model.fit`` runs per batch (SURVEY §3 call stacks).

    loss = model.loss(*batch)           (forward: librecsys_amd.so kernels via autograd)
    loss.backward()                     (kernels write weight grads in place into the arena)
                                        [DP, eager: <= 25 MB dense buckets all-reduced from
                                         autograd hooks as their gradients complete]
    grads += l1 sign(w) + 2 l2 w        (Keras kernel regularisers, rs_l1l2_grad)
    [DP] the regularised parameters' bucket (graph-captured DP: the whole flat gradient, one
         RCCL call), rank-ordered sparse exchange
         (owner-sharded tables: none -- their backward already pushed to the owners)
    dense Adam over the arena (one launch, zero_grad fused), sparse optimizer per table

Dense Adam follows tn.optimizer.Optimizer(tn.core.Adam(lr, .9, .999, 1e-8)) with tf.keras bias
correction (pinned); sparse tables use the optimizer they were created with.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr, stream_handle
from .embedding import is_sharded
from .layers import InteractingLayer
from .params import ParamArena

ARENA_ALIGN = 16  # floats: every layer's weights start 64-B aligned (the GEMMs' float4 path)


def exchange_sparse(table, pg, world, x_rows, x_grads):
    """Data-parallel sparse exchange of one table (dist.py protocol): compact -> all-gather ->
    merge in rank order."""
    from .dist import gather_sparse_lists
    cnt = table.n_touched[:1].clone()
    call("rs_sparse_compact", stream_handle(), ptr(table.grad), ptr(table.flag), ptr(table.touched),
         ptr(table.n_touched), table.dim, ptr(x_rows), ptr(x_grads), table.touched_cap)
    table.n_touched[:1].zero_()  # the count only: the completion words reset themselves and the
    # sticky overflow word n_touched[288] stays set until check_overflow reports it
    rows_all, grads_all, n = gather_sparse_lists(x_rows, x_grads, cnt, pg)
    for r in range(world if n else 0):
        call("rs_sparse_merge_rows", stream_handle(), ptr(rows_all[r]), ptr(grads_all[r]), n,
             table.dim, ptr(table.grad), ptr(table.flag), ptr(table.touched), ptr(table.n_touched),
             table.touched_cap)


class Trainer:
    """lr_groups: [(module, lr), ...] -- dense parameters of a sub-model with their own Adam
    learning rate (a joint workload whose towers the reference trains with separate
    tn.optimizer.Optimizer instances, e.g. config 5: staytime lr 5e-4 (staytime/model.py:72) and
    the DSSM lr 1e-4 (rough_rank/model.py:209)); every other parameter uses lr_dense.  Each group
    is a contiguous range of the arena with its own step counter (same count every step)."""

    def __init__(self, model, lr_dense: float, tables=(), process_group=None, beta1=0.9,
                 beta2=0.999, eps=1e-8, lr_groups=(), bucket_mb: float | None = None):
        self.model = model
        self.arena = ParamArena(model.parameters(), align=ARENA_ALIGN)
        dev = self.arena.data.device
        self.m = torch.zeros_like(self.arena.data)
        self.v = torch.zeros_like(self.arena.data)
        self.step_count = torch.zeros(1, device=dev, dtype=torch.int64)
        self.lr, self.b1, self.b2, self.eps = float(lr_dense), beta1, beta2, eps
        self.segments = self._lr_segments(lr_groups)
        # per segment: the completion counter of rs_dense_adam_done (its last block advances
        # the step counter) and the backward's seed (no ones_like fill launch per step)
        self._adam_done = [torch.zeros(288, device=dev, dtype=torch.int32) for _ in self.segments]
        self._seed = torch.ones((), device=dev)
        from .towers import register_unit_seed
        register_unit_seed(self._seed)  # the loss backward skips its multiply by this seed
        self.tables = list(tables)
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.regs = list(model.regularizers()) if hasattr(model, "regularizers") else []
        self.xbuf = {}
        self.on_dense_grad = None  # test hook: called with the exchanged flat dense gradient
        self._il_layers = [mod for mod in model.modules() if isinstance(mod, InteractingLayer)] \
            if hasattr(model, "modules") else []
        # eager DP: the dense all-reduce in buckets issued during backward (dist.BucketedAllReduce;
        # regularised parameters in the final bucket, after rs_l1l2_grad); bucket_mb <= 0: one
        # all-reduce after backward; None: sized from the arena (auto_bucket_bytes)
        self.bucketer = None
        if self.world > 1 and (bucket_mb is None or bucket_mb > 0):
            from .dist import BucketedAllReduce, auto_bucket_bytes
            nbytes = (auto_bucket_bytes(4 * self.arena.n) if bucket_mb is None
                      else int(bucket_mb * (1 << 20)))
            self.bucketer = BucketedAllReduce(self.arena, process_group, nbytes,
                                              late=[p for p, _, _ in self.regs])
        if self.world == 1:
            # single-GPU: tables that ask for it run in scan mode (pushes mark flags with plain
            # stores, no claims; the optimizer sweeps the flags) -- the DP exchange below needs
            # list mode's touched lists
            for t in self.tables:
                if getattr(t, "prefer_scan", False) and not t.deterministic:
                    t.mode = "scan"
        if self.world > 1:
            for t in self.tables:
                if is_sharded(t):
                    continue
                self.xbuf[id(t)] = (torch.empty(t.touched_cap, device=dev, dtype=torch.int32),
                                    torch.empty(t.touched_cap, t.dim, device=dev))

    def _lr_segments(self, lr_groups):
        """[(offset, n, lr, step counter)] covering the arena in order."""
        base = self.arena.data.data_ptr()
        ranges = []
        for mod, lr in lr_groups:
            offs = sorted(((p.data_ptr() - base) // 4, p.numel()) for p in mod.parameters())
            o0, end = offs[0][0], offs[0][0]
            for o, n in offs:
                if o < end or o - end >= ARENA_ALIGN:  # (alignment gaps between layers only)
                    raise ValueError("an lr group's parameters must be contiguous in the arena")
                end = o + n
            ranges.append((o0, end, float(lr)))
        ranges.sort()
        spans, k = [], 0
        for o0, o1, lr in ranges:
            if o0 < k:
                raise ValueError("lr groups overlap")
            if o0 > k:
                spans.append((k, o0, self.lr))
            spans.append((o0, o1, lr))
            k = o1
        if k < self.arena.n:
            spans.append((k, self.arena.n, self.lr))
        return [(o0, o1 - o0, lr, self.step_count if i == 0 else torch.zeros_like(self.step_count))
                for i, (o0, o1, lr) in enumerate(spans)]

    def step(self, *batch):
        # dropout masks: per-step host seeds restart at 0 each step and the device step counter
        # is added at run time (rs_set_seed_offset), so eager steps and graph replays draw the
        # same fresh mask per step
        for mod in self._il_layers:
            mod._calls = 0
        with _lib.seed_offset(self.step_count):
            return self._step(*batch)

    def _regularise(self):
        """All Keras kernel regularisers in one launch (rs_l1l2_grad_grouped, <= 16 per launch)."""
        s = stream_handle()
        for k0 in range(0, len(self.regs), 16):
            chunk = self.regs[k0:k0 + 16]
            n = len(chunk)
            wa, wp = _lib.c_array(ctypes.c_void_p, [ptr(p) for p, _, _ in chunk])
            ga, gp = _lib.c_array(ctypes.c_void_p, [ptr(p.grad) for p, _, _ in chunk])
            ca, cp = _lib.c_array(ctypes.c_int64, [p.numel() for p, _, _ in chunk])
            la, lp = _lib.c_array(ctypes.c_float, [float(l1) for _, l1, _ in chunk])
            ra, rp = _lib.c_array(ctypes.c_float, [float(l2) for _, _, l2 in chunk])
            call("rs_l1l2_grad_grouped", s, n, wp, gp, cp, lp, rp)

    def _backward(self, loss):
        """loss.backward with each replicated table's single-hot pushes issued as one grouped
        launch after the backward (SparseTable.begin_push_group; config 5: five pushes into the
        shared 10 M-row table -> one push + one claim launch)."""
        grp = [t for t in self.tables if not is_sharded(t) and hasattr(t, "begin_push_group")]
        for t in grp:
            t.begin_push_group()
        try:
            loss.backward(self._seed)
        except BaseException:
            for t in grp:
                t._deferred = None  # a failed backward pushes nothing
            raise
        for t in grp:
            t.end_push_group()

    def _step(self, *batch):
        loss = self.model.loss(*batch)
        if self.bucketer is not None:
            self.bucketer.arm(loss)  # buckets go out as backward produces their gradients
        self._backward(loss)
        if self.bucketer is not None:
            self.bucketer.finish(self._regularise)
        else:
            self._regularise()
        if self.world > 1:
            if self.bucketer is None:
                from .dist import allreduce_flat
                allreduce_flat(self.arena.grad, self.pg)
            for t in self.tables:
                if not is_sharded(t):
                    exchange_sparse(t, self.pg, self.world, *self.xbuf[id(t)])
        self._optimize(1.0 / self.world)
        return loss

    # ---- HIP-graph replay of whole steps (single GPU) --------------------------------------
    def _state(self):
        out = [self.arena.data, self.arena.grad, self.m, self.v]
        out += [cnt for *_, cnt in self.segments]
        for t in self.tables:
            out += [t.weight, t.grad, t.flag, t.n_touched, t.touched]
            out += [t.m, t.v] if hasattr(t, "m") else [t.g2sum]
        return out

    # ---- data parallel, graph-captured (capture_pool at world > 1) -----------------------
    # per step: graph A (forward, backward, regularisers, every replicated table's touched rows
    # compacted into its send list, the counts into dp_counts) -> eager collectives (the dense
    # all-reduce, ONE all-gather of all tables' counts, ONE host read of the per-table maxima,
    # one all-gather per table of nmax rows / gradient rows -- or, with dp_caps, fixed-size
    # all-gathers and no host read) -> graph B (rank-ordered merges that read the counts on the
    # device, rs_sparse_merge_rows_dev[_stride]; dense Adam; sparse optimizers).
    #
    # Owner-sharded tables route their lookups and pushes with all-to-alls INSIDE forward and
    # backward; with fixed routing (owner_cap, equal splits, no host read) those collectives are
    # captured into the forward/backward graph itself, which needs a backend whose collectives
    # are graph-capturable: RCCL ('nccl').  Their optimizer step is local (graph B).
    def _dp_setup(self, dp_caps=None):
        dev = self.arena.data.device
        self._rep = [t for t in self.tables if not is_sharded(t)]
        sharded = [t for t in self.tables if is_sharded(t)]
        if sharded:
            from .dist import uses_flat_all_gather
            if any(t.owner_cap is None for t in sharded):
                raise NotImplementedError(
                    "graph capture under DP with owner-sharded tables needs their fixed routing "
                    "(ShardedSparseTable(owner_cap=...) or Trainer.measure_dp_caps): variable "
                    "splits read the per-owner counts on the host inside the step")
            if not uses_flat_all_gather(self.pg):
                raise NotImplementedError(
                    "graph capture under DP with owner-sharded tables needs RCCL ('nccl'): the "
                    "tables' all-to-alls are captured into the forward/backward graph")
        T = len(self._rep)
        self.dp_counts = torch.zeros(max(T, 1), device=dev, dtype=torch.int32)
        self.dp_counts_all = torch.zeros(self.world * max(T, 1), device=dev, dtype=torch.int32)
        # sync-free exchange (dp_caps: rows per rank per step for each replicated table, e.g. the
        # batch's id count for that table -- a bound the caller knows): every rank's first cap
        # compacted rows travel whatever the counts, the merge reads the counts on the device
        # (rs_sparse_merge_rows_dev_stride) and a count past cap lands in dp_overflow
        # (check_dp_overflow, off the hot path).  None: one host read of the counts per step,
        # the all-gathers sized to the largest count.
        if dp_caps is not None:
            dp_caps = [int(min(c, t.touched_cap)) for c, t in zip(dp_caps, self._rep)]
            if len(dp_caps) != T or min(dp_caps, default=1) <= 0:
                raise ValueError("dp_caps: one positive row capacity per replicated table")
        self.dp_caps = dp_caps
        self.dp_overflow = torch.zeros(1, device=dev, dtype=torch.int32)
        self.dp_all = [(torch.empty(self.world * t.touched_cap, device=dev, dtype=torch.int32),
                        torch.empty(self.world * t.touched_cap * t.dim, device=dev))
                       for t in self._rep]

    def _dp_pack(self):
        s = stream_handle()
        for ti, t in enumerate(self._rep):
            rows, grads = self.xbuf[id(t)]
            self.dp_counts[ti:ti + 1].copy_(t.n_touched[:1])
            call("rs_sparse_compact", s, ptr(t.grad), ptr(t.flag), ptr(t.touched), ptr(t.n_touched),
                 t.dim, ptr(rows), ptr(grads), t.touched_cap)
            t.n_touched[:1].zero_()

    def _dp_exchange(self):
        from .dist import _all_gather_flat, allreduce_flat
        allreduce_flat(self.arena.grad, self.pg)
        if not self._rep:
            return
        _all_gather_flat(self.dp_counts_all, self.dp_counts, self.pg)
        if self.dp_caps is not None:  # fixed sizes: nothing read back on the host
            for ti, t in enumerate(self._rep):
                n = self.dp_caps[ti]
                rows, grads = self.xbuf[id(t)]
                rows_all, grads_all = self.dp_all[ti]
                _all_gather_flat(rows_all[:self.world * n], rows[:n], self.pg)
                _all_gather_flat(grads_all[:self.world * n * t.dim], grads[:n].reshape(-1), self.pg)
            return
        T = len(self._rep)
        nmax = self.dp_counts_all.view(self.world, T).max(0).values.tolist()  # the host sync
        for ti, t in enumerate(self._rep):
            n = int(nmax[ti])
            if n > t.touched_cap:
                raise RuntimeError(f"sparse exchange: {n} rows > touched capacity {t.touched_cap}")
            if n == 0:
                continue
            rows, grads = self.xbuf[id(t)]
            rows_all, grads_all = self.dp_all[ti]
            _all_gather_flat(rows_all[:self.world * n], rows[:n], self.pg)
            _all_gather_flat(grads_all[:self.world * n * t.dim], grads[:n].reshape(-1), self.pg)

    def _dp_merge_optimize(self):
        s = stream_handle()
        T = len(self._rep)
        for ti, t in enumerate(self._rep):
            rows_all, grads_all = self.dp_all[ti]
            for r in range(self.world):  # rank order -> identical sums on every replica
                if self.dp_caps is not None:
                    call("rs_sparse_merge_rows_dev_stride", s, ptr(rows_all), ptr(grads_all),
                         self.dp_counts_all.data_ptr() + 4 * ti, T, self.world, r,
                         self.dp_caps[ti], t.dim, ptr(t.grad), ptr(t.flag), ptr(t.touched),
                         ptr(t.n_touched), t.touched_cap, ptr(self.dp_overflow))
                    continue
                call("rs_sparse_merge_rows_dev", s, ptr(rows_all), ptr(grads_all),
                     self.dp_counts_all.data_ptr() + 4 * ti, T, self.world, r, t.touched_cap, t.dim,
                     ptr(t.grad), ptr(t.flag), ptr(t.touched), ptr(t.n_touched), t.touched_cap)
        self._optimize(1.0 / self.world)

    def _optimize(self, scale):
        s = stream_handle()
        if self.on_dense_grad is not None:
            self.on_dense_grad(self.arena.grad, scale)
        for (off, n, lr, cnt), done in zip(self.segments, self._adam_done):
            a = 4 * off
            call("rs_dense_adam_done", s, self.arena.data.data_ptr() + a,
                 self.arena.grad.data_ptr() + a, self.m.data_ptr() + a, self.v.data_ptr() + a, n,
                 ptr(cnt), lr, self.b1, self.b2, self.eps, scale, 1, ptr(done))
        for t in self.tables:
            t.step(grad_scale=scale)

    def _forward_backward(self, *batch):
        for mod in self._il_layers:
            mod._calls = 0
        with _lib.seed_offset(self.step_count):
            loss = self.model.loss(*batch)
            self._backward(loss)
        self._regularise()
        return loss

    def measure_dp_caps(self, batches, headroom: float = 1.25, quantum: int = 256):
        """dp_caps for capture_pool from the batches themselves: each batch's forward/backward
        runs once (eagerly; owner-sharded tables route with variable splits) and every
        replicated table's claimed-row count is read back; the per-table maximum over batches
        and ranks (one all-reduce MAX: every rank must use the same capacities), times
        ``headroom``, rounded up to ``quantum``, capped at the touched-list size.  Owner-sharded
        tables get their ``owner_cap`` set the same way from the largest number of ids one
        lookup sent to one owner (rounded up to quantum / 8).  The training state is restored
        afterwards.  A later step that touches more rows (or routes more ids) is caught by the
        sticky overflow words (step_pool reads them every dp_check_every replays), never trained
        on silently.  Returns the replicated tables' caps."""
        rep = [t for t in self.tables if not is_sharded(t)]
        sharded = [t for t in self.tables if is_sharded(t)]
        for t in sharded:
            t.owner_cap, t.peak_owner_ids = None, 0
        saved = [t.clone() for t in self._state()]
        peak = torch.zeros(max(len(rep) + len(sharded), 1), dtype=torch.int64)
        for b in batches:
            for t in rep:
                t.n_touched[:1].zero_()
            self._forward_backward(*b)
            for i, t in enumerate(rep):
                peak[i] = max(int(peak[i]), int(t.n_touched[0].item()))
            for t, v in zip(self._state(), saved):
                t.copy_(v)
        for i, t in enumerate(sharded):
            peak[len(rep) + i] = int(t.peak_owner_ids)
        if self.world > 1:
            pk = peak.to(self.arena.data.device)
            torch.distributed.all_reduce(pk, op=torch.distributed.ReduceOp.MAX, group=self.pg)
            peak = pk.cpu()
        torch.cuda.synchronize() if self.arena.data.is_cuda else None
        caps = []
        for i, t in enumerate(rep):
            c = -(-int(int(peak[i]) * headroom) // quantum) * quantum
            caps.append(int(min(max(c, quantum), t.touched_cap)))
        q8 = max(1, quantum // 8)
        for i, t in enumerate(sharded):
            c = -(-int(int(peak[len(rep) + i]) * headroom) // q8) * q8
            t.owner_cap = int(max(c, q8))
            t.route_stats.zero_()
        return caps

    def check_dp_overflow(self) -> None:
        """Raise if a sync-free DP step (capture_pool(dp_caps=...)) saw a rank touch more rows
        than its cap (rows lost in transit).  Reads the device: call it off the hot path."""
        n = int(self.dp_overflow.item()) if getattr(self, "dp_overflow", None) is not None else 0
        if n:
            self.dp_overflow.zero_()
            raise RuntimeError(f"sparse DP exchange overflow: a rank touched {n} rows, dp_caps "
                               f"{self.dp_caps} (raise dp_caps)")
        for t in self.tables:  # owner-sharded tables: ids past owner_cap in a fixed route
            if is_sharded(t) and t.owner_cap is not None:
                t.check_overflow()

    def capture_pool(self, batches, warmup: int = 1, dp_caps=None) -> None:
        """Record one whole training step per device-resident batch (forward, autograd backward,
        regularisers, dense Adam, sparse optimizer) into its own HIP graph; step_pool(i) replays
        batch i with no host work.  All graphs share one memory pool and are replayed in capture
        order (cyclic), which is what makes sharing it safe.  ``warmup`` eager steps run first
        (first-call allocations) and are rolled back, so capture changes no training state.
        Data parallel (world > 1): per batch a forward/backward graph (ending with the sparse
        lists packed), the collectives eager, then ONE merge + optimizer graph (_dp_* above);
        with dp_caps (per replicated table: rows one rank can touch per step) the collectives
        have fixed sizes and the host reads nothing back (sync-free; check_dp_overflow).
        Owner-sharded tables with fixed routing put their all-to-alls inside the forward/
        backward graph (RCCL only; _dp_setup)."""
        if self.world > 1:
            self._dp_setup(dp_caps)
        saved = [t.clone() for t in self._state()]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(warmup):
                self.step(*batches[i % len(batches)])
        torch.cuda.current_stream().wait_stream(side)
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        self.graphs, self.graph_loss = [], []
        from .dist import capture_error_mode
        mode = capture_error_mode()
        for b in batches:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                if self.world > 1:
                    loss = self._forward_backward(*b)
                    self._dp_pack()
                else:
                    loss = self.step(*b)
            self.graphs.append(g)
            self.graph_loss.append(loss.detach())
        self.graph_opt = None
        self._overflow_words = self._has_overflow_words()
        if self.world > 1:
            self.graph_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_opt, capture_error_mode=mode):  # allocates nothing
                self._dp_merge_optimize()
        # prime: replay each graph once and roll the state back (a graph's first launch after
        # capture is slower; AutoIntTrainer._prime_graphs)
        import os
        if not os.environ.get("RS_NO_GRAPH_PRIME"):
            saved = [t.clone() for t in self._state()]
            for g in self.graphs:
                g.replay()
            if self.graph_opt is not None:
                self.graph_opt.replay()
            torch.cuda.synchronize()
            for t, v in zip(self._state(), saved):
                t.copy_(v)
            torch.cuda.synchronize()

    # sync-free DP: the sticky overflow word is read back every this many replays (one host
    # read), so a run whose caps are too small stops within that many steps instead of training
    # on truncated sparse gradients
    dp_check_every = 256

    def _has_overflow_words(self) -> bool:
        """Whether a captured step can drop work silently: a fixed-capacity DP exchange
        (dp_caps) or an owner-sharded table with fixed routing (owner_cap), at any world size."""
        if getattr(self, "dp_caps", None) is not None:
            return True
        return any(is_sharded(t) and t.owner_cap is not None for t in self.tables)

    def step_pool(self, i: int):
        k = i % len(self.graphs)
        self.graphs[k].replay()
        if self.graph_opt is not None:
            self._dp_exchange()
            self.graph_opt.replay()
        if self._overflow_words:
            self._dp_replays = getattr(self, "_dp_replays", 0) + 1
            if self._dp_replays % self.dp_check_every == 0:
                self.check_dp_overflow()
        return self.graph_loss[k]

    def finish_pool(self) -> None:
        """Read the sticky overflow words once more (end of a replay run; raises like
        check_dp_overflow).  step_pool reads them every dp_check_every replays."""
        if self._has_overflow_words():
            self.check_dp_overflow()
