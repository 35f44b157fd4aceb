"""CPU, world_size 2 over gloo: the data-parallel exchange (dense bucket all-reduce, sparse list
all-gather + rank-ordered merge) gives identical results on every rank, equal to the single-
process sum over the union of the ranks' batches."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from recommendsystem_amd.dist import allreduce_flat, gather_sparse_lists, merge_reference

ROWS, DIM, CAP = 50, 4, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_lists(rank):
    """What rs_sparse_compact leaves on rank `rank`: unique rows + their local sums, -1 padded."""
    rng = np.random.default_rng(100 + rank)
    n = 7 + 5 * rank
    rows = rng.choice(ROWS, size=n, replace=False).astype(np.int32)
    grads = rng.normal(size=(n, DIM)).astype(np.float32)
    r = np.full(CAP, -1, np.int32)
    g = np.zeros((CAP, DIM), np.float32)
    r[:n], g[:n] = rows, grads
    return r, g, n


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dense = torch.arange(10, dtype=torch.float32) * (rank + 1)
    allreduce_flat(dense)
    r, g, n = _local_lists(rank)
    rows_all, grads_all, nmax = gather_sparse_lists(torch.from_numpy(r), torch.from_numpy(g),
                                                    torch.tensor([n], dtype=torch.int32))
    table = np.zeros((ROWS, DIM), np.float32)
    touched = merge_reference(rows_all.numpy(), grads_all.numpy(), table)
    out[rank] = (dense.numpy().copy(), table.copy(), sorted(touched), nmax)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_exchange_two_ranks():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    d0, t0, tc0, n0 = out[0]
    d1, t1, tc1, n1 = out[1]
    assert np.array_equal(d0, d1) and np.array_equal(d0, np.arange(10) * 3.0)
    assert np.array_equal(t0, t1) and tc0 == tc1  # replicas bitwise identical
    assert n0 == n1 == 12
    ref = np.zeros((ROWS, DIM), np.float64)
    for rank in range(world):
        r, g, n = _local_lists(rank)
        for k in range(n):
            ref[r[k]] += g[k]
    assert np.allclose(t0, ref, atol=1e-6)
    assert tc0 == sorted(set(int(v) for rank in range(world) for v in _local_lists(rank)[0] if v >= 0))


# ---- packed exchange (the AutoInt trainer's DP step: dist.exchange_packed) -------------------
N_DENSE, REC = 10, DIM + 1


def _packed_local(rank):
    """What the fused step leaves on rank `rank`: the dense bucket [grad | count | pad] and the
    packed records [row | grad] (rs_sparse_pack_scan's layout)."""
    r, g, n = _local_lists(rank)
    ld = (N_DENSE + 1 + 3) // 4 * 4
    send = torch.zeros(ld)
    send[:N_DENSE] = torch.arange(N_DENSE, dtype=torch.float32) * (rank + 1)
    send.view(torch.int32)[N_DENSE] = n
    recs = torch.zeros(CAP * REC)
    for u in range(n):
        recs[u * REC:(u + 1) * REC].view(torch.int32)[0] = int(r[u])
        recs[u * REC + 1:(u + 1) * REC] = torch.from_numpy(g[u])
    return send, recs, ld


def _packed_worker(rank, world, port, out):
    from recommendsystem_amd.dist import exchange_packed, merge_packed_reference
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    send, recs, ld = _packed_local(rank)
    recv = torch.zeros(world * ld)
    recs_all = torch.full((world * CAP * REC,), float("nan"))
    nmax = exchange_packed(send, recv, N_DENSE, recs, recs_all, REC)
    # the rank-ordered dense sum (what rs_partials_reduce_adam does over the gathered buckets)
    dense = recv.view(world, ld)[:, :N_DENSE].sum(0)
    table = np.zeros((ROWS, DIM), np.float32)
    touched = merge_packed_reference(recv, ld, N_DENSE, recs_all, REC, table)
    out[rank] = (dense.numpy().copy(), table.copy(), sorted(touched), nmax)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_packed_exchange_two_ranks():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_packed_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    d0, t0, tc0, n0 = out[0]
    d1, t1, tc1, n1 = out[1]
    assert np.array_equal(d0, d1) and np.array_equal(d0, np.arange(N_DENSE) * 3.0)
    assert np.array_equal(t0, t1) and tc0 == tc1  # replicas bitwise identical
    assert n0 == n1 == 12  # max(7, 12)
    ref = np.zeros((ROWS, DIM), np.float64)
    for rank in range(world):
        r, g, n = _local_lists(rank)
        for k in range(n):
            ref[r[k]] += g[k]
    assert np.allclose(t0, ref, atol=1e-6)
    assert tc0 == sorted(set(int(v) for rank in range(world) for v in _local_lists(rank)[0] if v >= 0))


def _packed_fixed_worker(rank, world, port, out):
    from recommendsystem_amd.dist import exchange_packed_fixed, merge_packed_reference
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    send, recs, ld = _packed_local(rank)
    recv = torch.zeros(world * ld)
    recs_all = torch.full((world * CAP * REC,), float("nan"))
    exchange_packed_fixed(send, recv, recs, recs_all, CAP, REC)  # no count read on the host
    table = np.zeros((ROWS, DIM), np.float32)
    touched = merge_packed_reference(recv, ld, N_DENSE, recs_all, REC, table, stride=CAP)
    out[rank] = (table.copy(), sorted(touched))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_packed_exchange_fixed_layout_two_ranks():
    """The sync-free exchange (every rank's whole capacity-sized record buffer, merged at stride
    cap) gives the same merged gradients as the count-sized one."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_packed_fixed_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (t0, tc0), (t1, tc1) = out[0], out[1]
    assert np.array_equal(t0, t1) and tc0 == tc1
    ref = np.zeros((ROWS, DIM), np.float64)
    for rank in range(world):
        r, g, n = _local_lists(rank)
        for k in range(n):
            ref[r[k]] += g[k]
    assert np.allclose(t0, ref, atol=1e-6)


def _packed_merged_worker(rank, world, port, out):
    from recommendsystem_amd.dist import (exchange_packed_merged, merge_packed_merged_reference,
                                          packed_layout)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    send, recs, _ = _packed_local(rank)
    ld, cap, S = packed_layout(N_DENSE, CAP, REC)
    assert ld % 4 == 0 and ld % REC == 0 and S % 4 == 0 and cap >= CAP
    buf = torch.full((S,), float("nan"))
    buf[:N_DENSE + 1] = send[:N_DENSE + 1]              # dense gradient + count
    buf[ld:ld + CAP * REC] = recs[:CAP * REC]
    buf_all = torch.zeros(world * S)
    exchange_packed_merged(buf, buf_all)               # ONE collective
    table = np.zeros((ROWS, DIM), np.float32)
    touched = merge_packed_merged_reference(buf_all, S, ld, N_DENSE, REC, table)
    dense = buf_all.view(world, S)[:, :N_DENSE].sum(0).numpy()
    out[rank] = (table.copy(), sorted(touched), dense)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_packed_exchange_merged_layout_two_ranks(world):
    """The AutoInt sync-free exchange as ONE all-gather of [dense | count | records] per rank
    (dist.packed_layout): the same merged gradients as the two-gather form (2 and 4 ranks)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_packed_merged_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    (t0, tc0, d0) = out[0]
    for r in range(1, world):
        t1, tc1, d1 = out[r]
        assert np.array_equal(t0, t1) and tc0 == tc1 and np.array_equal(d0, d1)
    ref = np.zeros((ROWS, DIM), np.float64)
    for rank in range(world):
        r, g, n = _local_lists(rank)
        for k in range(n):
            ref[r[k]] += g[k]
    assert np.allclose(t0, ref, atol=1e-6)
    dref = sum(_packed_local(r)[0][:N_DENSE] for r in range(world)).numpy()
    assert np.allclose(d0, dref, atol=1e-6)


class _Fn(torch.autograd.Function):
    """A kernel-style Function: writes its weight gradient IN PLACE into the arena and returns
    None for it (what the fused HIP kernels do), so only the node's saved W identifies it."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return x @ W

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        W.grad.add_(x.t() @ gy)
        return gy @ W.t(), None


def _bucket_worker(rank, world, port, out, late_mid=False, bucket_bytes=700):
    from torch import nn
    from recommendsystem_amd.dist import BucketedAllReduce
    from recommendsystem_amd.params import ParamArena
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)  # the same weights on every rank
    lin = [nn.Linear(16, 16) for _ in range(4)]
    Wk = nn.Parameter(torch.randn(16, 8) * 0.1)          # the in-place-writer's weight
    reg = nn.Parameter(torch.randn(8, 1) * 0.1)           # a 'late' (regularised) parameter
    # late_mid: the small late parameter (8 floats, under the arena's 16-float alignment gap)
    # sits between two early ones
    params = [p for l in lin for p in l.parameters()] + ([reg, Wk] if late_mid else [Wk, reg])
    arena = ParamArena(params)
    x = torch.randn(32, 16, generator=torch.Generator().manual_seed(10 + rank))

    def loss_fn():
        h = x
        for l in lin:
            h = torch.relu(l(h))
        return (_Fn.apply(h, Wk) @ reg).square().mean()

    # reference: whole backward, regulariser, one all-reduce of the arena
    arena.grad.zero_()
    loss_fn().backward()
    reg.grad.add_(0.01 * reg.detach())
    want = arena.grad.clone()
    dist.all_reduce(want)
    # bucketed: 700-B buckets (several per step), issued from the autograd hooks
    b = BucketedAllReduce(arena, bucket_bytes=bucket_bytes, late=[reg])
    arena.grad.zero_()
    loss = loss_fn()
    b.arm(loss)
    loss.backward()
    issued = b.issued_in_backward
    b.finish(lambda: reg.grad.add_(0.01 * reg.detach()))
    out[rank] = (arena.grad.numpy().copy(), want.numpy().copy(), issued, len(b.buckets))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_during_backward_two_ranks():
    """dist.BucketedAllReduce (the generic Trainer's eager DP step): buckets issued from autograd
    post-hooks during backward -- including a parameter whose gradient a kernel-style Function
    writes in place -- plus a late regularised bucket give exactly the one-bucket all-reduce
    (2 ranks: a + b either way), identical on both ranks."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, w0, issued0, nb = out[0]
    g1, w1, issued1, _ = out[1]
    assert nb > 2 and issued0 > 0 and issued0 == issued1
    assert np.array_equal(g0, w0) and np.array_equal(g1, w1) and np.array_equal(g0, g1)


def test_bucketed_allreduce_late_param_between_early_ones():
    """A small late (regularised) parameter between two early ones, 25 MB buckets: the bucket
    closes at the late parameter (a range spanning it would reduce its gradient during backward
    AND in finish(): world x the sum)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, _free_port(), out, True, 25 << 20), nprocs=world,
             join=True)
    g0, w0, _, nb = out[0]
    g1, w1, _, _ = out[1]
    assert nb == 2
    assert np.array_equal(g0, w0) and np.array_equal(g1, w1)


def _config5_bucket_worker(rank, world, port, out):
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd.workloads import StaytimeRoughRank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = StaytimeRoughRank(rows=1001, device="cpu", seed=0)  # config 5's dense towers
    trn = Trainer(m, 5e-4, [m.table], process_group=dist.group.WORLD,
                  lr_groups=[(m.dssm, m.rr_cfg.lr_dense)])   # default bucket size
    params = list(m.parameters())
    g = torch.Generator().manual_seed(100 + rank)
    coef = [torch.randn(p.shape, generator=g) for p in params]

    def loss_fn():  # every parameter in registration order: backward meets them in reverse
        tot = torch.zeros(())
        for p, c in zip(params, coef):
            tot = tot + (p * c).sum()
        return tot

    trn.arena.grad.zero_()
    loss_fn().backward()
    want = trn.arena.grad.clone()
    dist.all_reduce(want)
    trn.arena.grad.zero_()
    loss = loss_fn()
    trn.bucketer.arm(loss)
    loss.backward()
    issued = trn.bucketer.issued_in_backward
    trn.bucketer.finish()
    out[rank] = (trn.arena.grad.numpy().copy(), want.numpy().copy(), issued,
                 len(trn.bucketer.buckets), 4 * trn.arena.n)
    dist.barrier()
    dist.destroy_process_group()


def test_config5_arena_buckets_issue_during_backward():
    """The config-5 (staytime + rough_rank) dense arena with the Trainer's default bucket size
    (dist.auto_bucket_bytes: ~1/4 of the arena): several buckets, more than one of them issued
    from the autograd hooks while backward still runs, and the result equals one flat
    all-reduce."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_config5_bucket_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, w0, issued, nb, nbytes = out[0]
    g1, w1, _, _, _ = out[1]
    assert nbytes > 10 << 20 and nb >= 4 and issued > 1, (nbytes, nb, issued)
    assert np.array_equal(g0, w0) and np.array_equal(g1, w1)
