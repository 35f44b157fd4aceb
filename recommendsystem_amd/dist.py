"""Data-parallel gradient exchange: one process per GPU, torch.distributed with the
'nccl' backend (= RCCL over xGMI on ROCm).  Replaces tensornet's dense MPI all-reduce
(tn.optimizer.Optimizer) and its PS sparse push (tn.layers.EmbeddingFeatures) for DP training.

  dense  : the model's flat gradient arena.  AutoInt: the packed exchange below (all-gathered
           buckets summed in rank order, 15.4 K floats).  The generic Trainer's eager DP step:
           BucketedAllReduce -- arena ranges of <= 25 MB issued as async all-reduces from
           autograd post-hooks while the rest of backward runs; its graph-captured DP step: one
           all-reduce of the whole arena after the captured forward / backward.
  sharded: owner-sharded tables (embedding.ShardedSparseTable, row owner = row % world) move
           lookups and gradients with two all-to-alls each way instead: variable splits
           (all_to_all_v; counts first, read on the host) or, with owner_cap, equal fixed-size
           blocks (all_to_all_fixed; no host read, graph-capturable under RCCL).
  sparse : each rank pre-reduces its touched rows locally (rs_sparse_grad_accumulate), compacts
           them into (rows, grads) lists, the lists are all-gathered (counts first, then lists
           padded to the max count with row -1), and every rank merges the lists IN RANK ORDER
           with atomic-free adds (rs_sparse_merge_rows): identical inputs + identical order ->
           bitwise-identical sparse updates on every replica.

The transport functions are device-agnostic (gloo on CPU tensors in tests/test_dist.py, RCCL
on the GPU box); the merge itself runs in librecsys_amd.so.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def capture_error_mode() -> str:
    """HIP-graph capture mode for the trainers: "thread_local" whenever an RCCL process group
    exists.  Its watchdog thread polls the events of earlier (eager) collectives with
    hipEventQuery, which a global-mode capture forbids process-wide (hipErrorStreamCaptureUnsupported
    -> the watchdog aborts the process); thread-local mode restricts only the capturing thread.
    Otherwise torch's default ("global")."""
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        return "thread_local"
    return "global"


def allreduce_flat(grad: torch.Tensor, group=None) -> None:
    """Sum the flat dense gradient over ranks in place (the optimizer scales by 1/world)."""
    dist.all_reduce(grad, group=group)


def gather_sparse_lists(rows: torch.Tensor, grads: torch.Tensor, count: torch.Tensor, group=None):
    """All-gather every rank's compacted (rows, grads) list.

    rows [cap] int32 (-1 padded past `count`), grads [cap, dim], count [1] int32.
    Returns (rows_all [world, n], grads_all [world, n, dim], n) with n = max count (n == 0 ->
    nothing touched anywhere).  The host learns n through one small all-gather.
    """
    world = dist.get_world_size(group)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count, group=group)
    n = int(torch.stack(counts).max().item())
    if n == 0:
        return None, None, 0
    rows_all = torch.empty(world, n, dtype=rows.dtype, device=rows.device)
    grads_all = torch.empty(world, n, grads.shape[1], dtype=grads.dtype, device=grads.device)
    dist.all_gather(list(rows_all.unbind(0)), rows[:n].contiguous(), group=group)
    dist.all_gather(list(grads_all.unbind(0)), grads[:n].contiguous(), group=group)
    return rows_all, grads_all, n


def _all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out[r * inp.numel():(r + 1) * inp.numel()] = rank r's inp (one contiguous receive buffer).
    RCCL ('nccl') moves it with one all_gather_into_tensor; gloo gets per-rank views.  The path
    is chosen by backend, never by catching a failure (a failed collective on one rank must not
    turn into a different collective on it while the others wait in the first)."""
    if uses_flat_all_gather(group):
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        world = dist.get_world_size(group)
        dist.all_gather(list(out.view(world, -1).unbind(0)), inp, group=group)


def uses_flat_all_gather(group=None) -> bool:
    """True for RCCL ('nccl' on ROCm), the backend with a flat all_gather_into_tensor."""
    return dist.get_backend(group) == "nccl"


def exchange_packed(send: torch.Tensor, recv: torch.Tensor, n_dense: int, recs: torch.Tensor,
                    recs_all: torch.Tensor, rec_floats: int, group=None) -> int:
    """The AutoInt trainer's data-parallel exchange: TWO all-gathers per step.

    send  [ld] fp32 : this rank's dense gradient (n_dense floats) + its record count (int32 bits
                      at index n_dense), ld >= n_dense + 1;
    recv  [world * ld] : every rank's send buffer (a deterministic rank-ordered sum of the dense
                      part replaces the all-reduce, so replicas stay bitwise identical);
    recs  [cap * rec_floats] : this rank's packed sparse records (rs_sparse_pack_scan);
    recs_all [world * cap * rec_floats] : receives nmax records per rank, rank r's at
                      r * nmax * rec_floats (rs_sparse_merge_packed recomputes nmax on the device).
    Returns nmax = the largest count (the only host synchronisation of the step).
    """
    world = dist.get_world_size(group)
    ld = send.numel()
    _all_gather_flat(recv, send, group)
    counts = recv.view(torch.int32).view(world, ld)[:, n_dense]
    nmax = int(counts.max().item())
    if nmax > 0:
        k = nmax * rec_floats
        _all_gather_flat(recs_all[:world * k], recs[:k], group)
    return nmax


def exchange_packed_fixed(send: torch.Tensor, recv: torch.Tensor, recs: torch.Tensor,
                          recs_all: torch.Tensor, cap: int, rec_floats: int, group=None) -> None:
    """exchange_packed without the host synchronisation: every rank's WHOLE record buffer (cap
    records, cap = the most rows one rank can touch per step, so it never overflows) is
    all-gathered, rank r's at r * cap * rec_floats, and the merge (rs_sparse_merge_packed_stride)
    reads each rank's count on the device.  More bytes on the links (cap instead of the largest
    count), no host read: the CPU enqueues the next step while this one runs."""
    world = dist.get_world_size(group)
    k = cap * rec_floats
    _all_gather_flat(recv, send, group)
    _all_gather_flat(recs_all[:world * k], recs[:k], group)


def packed_layout(n_dense: int, cap: int, rec_floats: int):
    """The merged send buffer of the sync-free AutoInt exchange: ONE all-gather per step.

    [dense gradient (n_dense) | record count (int32 bits) | pad | records (cap x rec_floats)]
    ld (the dense part) is rounded up to a multiple of lcm(4, rec_floats) and cap to a multiple
    of 4, so the per-rank block S = ld + cap * rec_floats keeps 16-B row alignment for the dense
    sum and every rank's records start on a record boundary: in the gathered buffer rank r's
    records are at (r * S + ld) floats = record (r * S + ld) / rec_floats, i.e. a record stride
    of S / rec_floats per rank (rs_sparse_merge_packed_stride).  Returns (ld, cap, S)."""
    import math
    q = 4 * rec_floats // math.gcd(4, rec_floats)
    ld = -(-(n_dense + 1) // q) * q
    cap = -(-cap // 4) * 4
    return ld, cap, ld + cap * rec_floats


def exchange_packed_merged(buf: torch.Tensor, buf_all: torch.Tensor, group=None) -> None:
    """exchange_packed_fixed in ONE collective: every rank's whole packed_layout buffer (dense
    gradient, count, capacity-sized records) all-gathered into buf_all [world * S] -- half the
    collective launches of the two-gather form, no host read."""
    _all_gather_flat(buf_all, buf, group)


def merge_packed_merged_reference(buf_all, S, ld, n_dense, rec_floats, table_grad):
    """Host restatement of the merges over the merged layout (CPU tests): rank r's count at
    r * S + n_dense, its records from r * S + ld."""
    world = buf_all.numel() // S
    counts = buf_all.view(torch.int32).view(world, S)[:, n_dense].tolist()
    touched = []
    for r in range(world):
        for u in range(counts[r]):
            off = r * S + ld + u * rec_floats
            rec = buf_all[off:off + rec_floats]
            row = int(rec[:1].view(torch.int32)[0])
            if row not in touched:
                touched.append(row)
            table_grad[row] += rec[1:].numpy()
    return touched


def merge_packed_reference(recv, ld, n_dense, recs_all, rec_floats, table_grad, stride=0):
    """Host restatement of rs_sparse_merge_packed (stride 0: rank r's records at r * nmax) /
    rs_sparse_merge_packed_stride (at r * stride) over every rank in order (CPU tests)."""
    world = recv.numel() // ld
    counts = recv.view(torch.int32).view(world, ld)[:, n_dense].tolist()
    nmax = max(counts)
    touched = []
    for r in range(world):
        base = r * (stride if stride > 0 else nmax) * rec_floats
        for u in range(counts[r]):
            rec = recs_all[base + u * rec_floats: base + (u + 1) * rec_floats]
            row = int(rec[:1].view(torch.int32)[0])
            if row not in touched:
                touched.append(row)
            table_grad[row] += rec[1:].numpy()
    return touched


def merge_reference(rows_all, grads_all, table_grad):
    """Host restatement of the rank-ordered merge (what rs_sparse_merge_rows does per rank),
    used by the CPU tests: table_grad[row] += grads in rank order, skipping -1 padding."""
    touched = []
    for r in range(rows_all.shape[0]):
        for u in range(rows_all.shape[1]):
            row = int(rows_all[r, u])
            if row < 0:
                continue
            if row not in touched:
                touched.append(row)
            table_grad[row] += grads_all[r, u]
    return touched


def all_to_all_v(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None) -> None:
    """Variable-split all-to-all along dim 0 (rank r's slice of inp goes to rank r; out holds the
    slices from ranks 0..world-1 in rank order).  RCCL moves device tensors directly; gloo stages
    device tensors through host memory (backend chosen by name, as in _all_gather_flat)."""
    if inp.is_cuda and dist.get_backend(group) != "nccl":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), list(out_splits), list(in_splits), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=group)


def all_to_all_fixed(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """Equal-split all-to-all along dim 0 (world blocks of inp.shape[0] / world rows): the
    fixed-capacity routing of owner-sharded tables.  Nothing host-side depends on the data, so
    under RCCL it can be captured in a HIP graph; gloo stages device tensors through the host."""
    if inp.is_cuda and dist.get_backend(group) != "nccl":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=group)


def exchange_counts(counts: torch.Tensor, group=None):
    """counts [world] int32 (ids this rank sends to each owner) -> (send_splits, recv_splits) as
    host lists: one 1-element-per-rank all-to-all and the step's host synchronisation."""
    world = counts.numel()
    recv = torch.empty_like(counts)
    all_to_all_v(recv, counts, [1] * world, [1] * world, group)
    return counts.tolist(), recv.tolist()


def auto_bucket_bytes(arena_bytes: int) -> int:
    """Default dense bucket for an arena of arena_bytes: about a quarter of it, between 1 MB and
    25 MB -- several buckets for the configs-3/5 arenas (2.2 MB -> 1 MB, 13.9 MB -> 3.5 MB), so
    the first ones go out while backward still runs, yet each all-reduce stays large enough for
    the per-link bandwidth of xGMI (ring collectives pay a fixed latency per call)."""
    return int(min(25 << 20, max(1 << 20, arena_bytes // 4)))


class BucketedAllReduce:
    """The flat dense gradient all-reduced in buckets issued DURING backward (SURVEY §8(e):
    "buckets of <= 25 MB, launched as backward produces the grads"; the reference's
    tn.optimizer.Optimizer(dense_opt) at staytime/model.py:89, rough_rank/model.py:220 syncs the
    dense gradients through tensornet's MPI allreduce after the whole backward).

    Buckets are contiguous ranges of the parameter arena, built from its END (the parameters a
    model registers last produce their gradients first in backward), each <= bucket_bytes.
    ``arm(loss)`` walks loss's autograd graph once per step and registers a post-hook on every
    node that produces an arena parameter's gradient: its AccumulateGrad node, and every custom
    kernel Function node that saved the parameter (the fused kernels write weight gradients in
    place and return None for them).  A parameter is ready when all its producer nodes have run;
    a bucket is issued (async all_reduce, SUM, in place) once its parameters are ready AND every
    earlier bucket has been issued -- the same collective order on every rank.  The hooks run on
    the host as the autograd engine finishes each node, i.e. after that node's kernels are
    enqueued: the collective is ordered after them on the device and overlaps the backward
    kernels enqueued later.  ``late`` parameters (regularised ones: rs_l1l2_grad completes their
    gradient after backward) go to the final bucket, issued by ``finish`` after the caller's
    completion step; ``finish`` also issues buckets whose parameters got no gradient this step
    (their zeros still take part) and waits for everything."""

    def __init__(self, arena, group=None, bucket_bytes: int = 25 << 20, late=()):
        self.arena, self.group = arena, group
        base = arena.data.data_ptr()
        late_ids = {id(p) for p in late}
        spans = []  # (offset, numel, param)
        for p in arena.params:
            spans.append(((p.data_ptr() - base) // 4, p.numel(), p))
        spans.sort(key=lambda t: t[0])
        cap = max(1, int(bucket_bytes) // 4)
        self.buckets = []   # [(off, n, [params])] in issue order
        cur, cur_lo, cur_hi = [], None, None
        for off, n, p in reversed(spans):
            if id(p) in late_ids:
                # a late parameter between two early ones ends the bucket: a range spanning it
                # would all-reduce its gradient during backward (racing rs_l1l2_grad) and again
                # in finish()
                if cur:
                    self.buckets.append((cur_lo, cur_hi - cur_lo, cur))
                    cur, cur_lo, cur_hi = [], None, None
                continue
            # adjacent in the arena up to its layer-alignment gap (< 16 floats of zeros)
            contiguous = cur_lo is None or 0 <= cur_lo - (off + n) < 16
            if cur and (not contiguous or cur_hi - off > cap):
                self.buckets.append((cur_lo, cur_hi - cur_lo, cur))
                cur, cur_lo, cur_hi = [], None, None
            cur.append(p)
            cur_hi = off + n if cur_hi is None else cur_hi
            cur_lo = off
        if cur:
            self.buckets.append((cur_lo, cur_hi - cur_lo, cur))
        self.late = [(off, n, p) for off, n, p in spans if id(p) in late_ids]
        self._param_bucket = {}
        for k, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self._param_bucket[id(p)] = k
        self._by_ptr = {}
        for off, n, p in spans:
            self._by_ptr[p.data_ptr()] = p
        self._handles = []
        self.issued_in_backward = 0  # diagnostics / tests: buckets issued by the hooks

    # -- per step ---------------------------------------------------------------------------
    def arm(self, loss: torch.Tensor) -> None:
        self._handles = []
        self._next = 0
        self.issued_in_backward = 0
        self._pending = [0] * len(self.buckets)      # unready params per bucket
        self._producers = {}                         # id(param) -> producer nodes left
        seen, stack = set(), [loss.grad_fn] if loss.grad_fn is not None else []
        node_params = []
        while stack:
            node = stack.pop()
            if node is None or node in seen:
                continue
            seen.add(node)
            ps = self._node_params(node)
            if ps:
                node_params.append((node, ps))
            for nxt, _ in node.next_functions:
                if nxt is not None:
                    stack.append(nxt)
        for node, ps in node_params:
            for p in ps:
                self._producers[id(p)] = self._producers.get(id(p), 0) + 1
            node.register_hook(self._make_hook(ps))
        for pid, _ in self._producers.items():
            k = self._param_bucket.get(pid)
            if k is not None:
                self._pending[k] += 1

    def _node_params(self, node):
        out = []
        var = getattr(node, "variable", None)  # AccumulateGrad
        if var is not None:
            p = self._by_ptr.get(var.data_ptr())
            if p is not None and id(p) in self._param_bucket:
                out.append(p)
            return out
        try:
            saved = node.saved_tensors  # custom (kernel) Functions
        except (AttributeError, RuntimeError):
            return out
        for t in saved:
            if t is None:
                continue
            p = self._by_ptr.get(t.data_ptr())
            if p is not None and p.numel() == t.numel() and id(p) in self._param_bucket:
                out.append(p)
        return out

    def _make_hook(self, ps):
        def hook(*_):
            for p in ps:
                pid = id(p)
                self._producers[pid] -= 1
                if self._producers[pid] == 0:
                    self._pending[self._param_bucket[pid]] -= 1
            self._issue_ready()
        return hook

    def _issue(self, k):
        off, n, _ = self.buckets[k]
        self._handles.append(dist.all_reduce(self.arena.grad[off:off + n], group=self.group,
                                             async_op=True))

    def _issue_ready(self):
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            self._issue(self._next)
            self._next += 1
            self.issued_in_backward += 1

    def finish(self, complete_late=None) -> None:
        """After backward: issue what is left (buckets without gradients this step), run
        complete_late() (the regularisers) and issue the late parameters' bucket, wait."""
        while self._next < len(self.buckets):
            self._issue(self._next)
            self._next += 1
        if complete_late is not None:
            complete_late()
        if self.late:
            lo = min(off for off, _, _ in self.late)
            hi = max(off + n for off, n, _ in self.late)
            # one range covering the late parameters (gaps belong to early buckets, already
            # being reduced: the late range must not overlap them)
            if hi - lo == sum(n for _, n, _ in self.late):
                self._handles.append(dist.all_reduce(self.arena.grad[lo:hi], group=self.group,
                                                     async_op=True))
            else:
                for off, n, _ in self.late:
                    self._handles.append(dist.all_reduce(self.arena.grad[off:off + n],
                                                         group=self.group, async_op=True))
        for h in self._handles:
            h.wait()
        self._handles = []
