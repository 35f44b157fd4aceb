"""N2 owner-sharded tables on CPU (gloo, world size 2): the routing oracle, and the host
choreography of embedding.ShardedSparseTable (count exchange, variable-split all-to-alls, the
gather / scatter / push order) with the five device kernels it calls replaced by host
restatements, so the collective protocol is checked here; tests/test_gpu_sharded.py runs the
real kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ctr_oracle as npo


def test_owner_route_oracle():
    rows = np.array([7, -1, 4, 9, 2, 11, 3, 100, 0, 5], dtype=np.int64)
    sl, sp, c = npo.owner_route(rows, 3, 12)
    # owners: 7->1 4->1 9->0 2->2 11->2 3->0 0->0 5->2; -1 and 100 (>= 12 rows) dropped
    assert c.tolist() == [3, 2, 3]
    assert sp.tolist() == [3, 6, 8, 0, 2, 4, 5, 9]          # stable within each owner
    assert sl.tolist() == [3, 1, 0, 2, 1, 0, 3, 1]          # row // 3
    sl, sp, c = npo.owner_route(np.array([], dtype=np.int64), 4, 10)
    assert sl.size == 0 and c.tolist() == [0, 0, 0, 0]


# ---- host restatements of the kernels ShardedSparseTable drives (pointer args are tensors) ----
def _host_call(name, *a):
    if name == "rs_owner_route":
        _, rows, n, world, table_rows, send_local, send_pos, counts, _ws, _wn = a
        sl, sp, c = npo.owner_route(rows.numpy(), world, table_rows)
        send_local[:sl.size] = torch.from_numpy(sl)
        send_pos[:sp.size] = torch.from_numpy(sp)
        counts.copy_(torch.from_numpy(c))
    elif name == "rs_owner_route_fixed":
        _, rows, n, world, table_rows, cap, send_local, slot, stats, _ws, _wn = a
        sl, st, peak = npo.owner_route_fixed(rows.numpy(), world, table_rows, cap)
        send_local.copy_(torch.from_numpy(sl))
        slot.copy_(torch.from_numpy(st))
        stats[0] = max(int(stats[0]), peak)
    elif name == "rs_gather_rows":
        _, src, src_ld, idx, n, dim, dst, dst_ld = a
        s = src.reshape(-1, src_ld)[:, :dim]
        i = idx.long()
        dst.reshape(-1, dst_ld)[:n, :dim] = torch.where((i >= 0)[:, None], s[i.clamp(min=0)], 0.0)
    elif name == "rs_scatter_rows":
        _, src, src_ld, idx, n, dim, dst, dst_ld = a
        i = idx.long()
        ok = i >= 0
        dst.reshape(-1, dst_ld)[i[ok], :dim] = src.reshape(-1, src_ld)[:n][ok, :dim]
    elif name == "rs_segment_expand":
        _, dout, ld, fs, offsets, B, F, comb, dim, dE = a
        o = offsets.long()
        for s in range(B * F):
            b, f = divmod(s, F)
            k0, k1 = int(o[s]), int(o[s + 1])
            sc = float(npo.combiner_scale(k1 - k0, ["sum", "mean", "sqrtn"][comb]))
            dE[k0:k1] = sc * dout.reshape(-1)[b * ld + f * fs: b * ld + f * fs + dim]
    elif name == "rs_embedding_lookup_fwd":
        _, ids, offsets, B, F, row_base, bucket, hm, comb, table, trows, dim, out, ld, fs, rows_out = a
        n = ids.numel()
        if offsets is None:
            fields = np.tile(np.arange(F), B)
        else:
            seg = np.repeat(np.arange(B * F), np.diff(offsets.numpy()))
            fields = seg % F
        rows = npo.hash_rows(ids.numpy().reshape(-1), fields, row_base.numpy(), bucket.numpy(),
                             ["mod", "splitmix"][hm])
        if table is None:
            rows_out.copy_(torch.from_numpy(np.where(rows < trows, rows, -1).astype(np.int32)))
            return 0
        W = table.reshape(-1, dim).numpy()
        offs = offsets.numpy() if offsets is not None else np.arange(n + 1)
        e, _ = npo.embedding_lookup(ids.numpy().reshape(-1), offs, B, F, row_base.numpy(),
                                    bucket.numpy(), W, ["mod", "splitmix"][hm],
                                    ["sum", "mean", "sqrtn"][comb])
        out.reshape(B, F, dim).copy_(torch.from_numpy(e.astype(np.float32)))
    elif name == "rs_sequence_lookup_fwd":
        _, ids, offsets, B, T, rb, bk, hm, table, dim, out, ss, rs, mask, mld, lengths, rows_out = a
        assert table is None
        _, m, r = npo.sequence_lookup(ids.numpy(), offsets.numpy(), B, T, rb, bk,
                                      np.zeros((rb + bk, 4), np.float32), ["mod", "splitmix"][hm])
        rows_out.copy_(torch.from_numpy(r.reshape(-1).astype(np.int32)))
        mask.copy_(torch.from_numpy(m.astype(np.uint8)))
        lengths.copy_(torch.from_numpy(m.sum(1).astype(np.int32)))
    elif name in ("rs_sparse_grad_accumulate", "rs_sparse_grad_accumulate_ws"):
        _, rows, offsets, B, F, dout, ld, fs, dim, comb, grad, flag, touched, n_t, cap = a[:15]
        assert offsets is None and F == 1
        r = rows.long()
        ok = r >= 0
        grad.index_add_(0, r[ok], dout.reshape(-1, ld)[:, :dim][ok])
        flag[r[ok]] = -2
    else:
        raise AssertionError(f"unexpected kernel {name}")
    return 0


def _patch():
    from recommendsystem_amd import _lib, embedding
    embedding.call = _host_call
    embedding.ptr = lambda t: t
    embedding.stream_handle = lambda: None
    _lib.require_device = lambda *t: None
    embedding.ShardedSparseTable._workspace = lambda self, n: torch.empty(0, dtype=torch.uint8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ROWS, DIM, WORLD = 103, 8, 2


def _batch(rank):
    rng = np.random.default_rng(70 + rank)
    B, F = 6, 3
    lens = rng.integers(0, 4, size=B * F)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ids = rng.integers(0, 10_000, size=int(offs[-1])).astype(np.int64)
    single = rng.integers(0, 10_000, size=(B, F)).astype(np.int64)
    slens = rng.integers(0, 6, size=B)
    soffs = np.concatenate([[0], np.cumsum(slens)]).astype(np.int32)
    sids = rng.integers(0, 10_000, size=int(soffs[-1])).astype(np.int64)
    return [torch.from_numpy(x) for x in (ids, offs, single, sids, soffs)]


def _worker(rank, world, port, out, owner_cap=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch()
    from recommendsystem_amd import dist as rdist
    from recommendsystem_amd.embedding import (EmbeddingFeatures, SequenceEmbedding,
                                               ShardedSparseTable, SparseAdaGrad)
    t = ShardedSparseTable(ROWS, DIM, SparseAdaGrad(), device="cpu", seed=4,
                           process_group=dist.group.WORLD, owner_cap=owner_cap)
    if owner_cap is not None:  # fixed routing: no count exchange may run
        rdist.exchange_counts = None
    ids, offs, single, sids, soffs = _batch(rank)
    var = EmbeddingFeatures(t, [50, 40, 13], combiner="mean", hash_mode="splitmix")
    one = EmbeddingFeatures(t, [ROWS] * 3, row_base=[0] * 3, combiner="sum", hash_mode="splitmix")
    seq = SequenceEmbedding(t, ROWS, 4, hash_mode="splitmix")
    ev = var(ids, offs)
    eo = one(single)
    es, mask = seq(sids, soffs)
    gen = torch.Generator().manual_seed(rank)
    dv, do, ds = (torch.randn(x.shape, generator=gen) for x in (ev, eo, es))
    torch.autograd.backward([ev, eo, es], [dv, do, ds])
    overflow = None
    if owner_cap is not None:
        try:
            t.check_overflow()
        except RuntimeError as e:
            overflow = str(e)
    out[rank] = dict(ev=ev.detach().numpy(), eo=eo.detach().numpy(), es=es.detach().numpy(),
                     mask=mask.numpy(), dv=dv.numpy(), do=do.numpy(), ds=ds.numpy(),
                     grad=t.grad.numpy().copy(), local_rows=t.weight.shape[0], overflow=overflow)
    dist.barrier()
    dist.destroy_process_group()


def test_owner_route_fixed_oracle():
    rows = np.array([7, -1, 4, 9, 2, 11, 3, 100, 0, 5], dtype=np.int64)
    sl, slot, peak = npo.owner_route_fixed(rows, 3, 12, 2)
    # owner 0: 9, 3, 0 (0 past cap 2); owner 1: 7, 4; owner 2: 2, 11, 5 (5 past cap)
    assert peak == 3
    assert sl.tolist() == [3, 1, 2, 1, 0, 3]
    assert slot.tolist() == [2, -1, 3, 0, 4, 5, 1, -1, -1, -1]
    sl, slot, peak = npo.owner_route_fixed(np.array([], dtype=np.int64), 2, 10, 3)
    assert sl.tolist() == [-1] * 6 and slot.size == 0 and peak == 0


@pytest.mark.parametrize("owner_cap", [None, 64])
def test_sharded_table_protocol_world2(owner_cap):
    """owner_cap: the sync-free fixed routing (equal-split all-to-alls, no count exchange); 64
    ids per (requester, owner) per lookup holds every lookup here, so the results are the same."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(WORLD, _free_port(), out, owner_cap), nprocs=WORLD, join=True)
    from recommendsystem_amd.embedding import SparseAdaGrad, SparseTable
    W = SparseTable.initial_weight(ROWS, DIM, SparseAdaGrad(), 0.05, 4).numpy().astype(np.float64)
    assert out[0]["local_rows"] == 52 and out[1]["local_rows"] == 51
    gsum = np.zeros((ROWS, DIM))
    for r in range(WORLD):
        ids, offs, single, sids, soffs = [x.numpy() for x in _batch(r)]
        o = out[r]
        rb_var = np.array([0, 50, 90])
        ev, _ = npo.embedding_lookup(ids, offs, 6, 3, rb_var, [50, 40, 13], W, "splitmix", "mean")
        np.testing.assert_allclose(o["ev"], ev, rtol=1e-6, atol=1e-7)
        eo, _ = npo.embedding_lookup(single.reshape(-1), np.arange(19), 6, 3, np.zeros(3, np.int64),
                                     [ROWS] * 3, W, "splitmix", "sum")
        np.testing.assert_allclose(o["eo"], eo, rtol=1e-6, atol=1e-7)
        es, m, srows = npo.sequence_lookup(sids, soffs, 6, 4, 0, ROWS, W, "splitmix")
        np.testing.assert_allclose(o["es"], es, rtol=1e-6, atol=1e-7)
        assert np.array_equal(o["mask"], m)
        # every id's gradient, summed at its row over both ranks
        seg = np.repeat(np.arange(18), np.diff(offs))
        rv = npo.hash_rows(ids, seg % 3, rb_var, [50, 40, 13], "splitmix")
        cnt = np.diff(offs)[seg]
        np.add.at(gsum, rv, o["dv"].reshape(18, DIM)[seg] / cnt[:, None])
        ro = npo.hash_rows(single.reshape(-1), np.tile(np.arange(3), 6), np.zeros(3, np.int64),
                           [ROWS] * 3, "splitmix")
        np.add.at(gsum, ro, o["do"].reshape(-1, DIM))
        ok = srows.reshape(-1) >= 0
        np.add.at(gsum, srows.reshape(-1)[ok], o["ds"].reshape(-1, DIM)[ok])
    for r in range(WORLD):  # owner r holds rows r, r + 2, ...
        np.testing.assert_allclose(out[r]["grad"], gsum[r::WORLD], rtol=1e-5, atol=1e-6)
        assert out[r]["overflow"] is None


def test_sharded_fixed_routing_overflow_is_reported():
    """A lookup that sends more ids to one owner than owner_cap drops the excess and the sticky
    route word makes check_overflow raise (never trained on silently)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(WORLD, _free_port(), out, 4), nprocs=WORLD, join=True)
    for r in range(WORLD):
        assert out[r]["overflow"] is not None and "owner_cap is 4" in out[r]["overflow"]


def test_initial_shard_equals_slice_of_full_table():
    """ShardedSparseTable draws only its own rows (row chunks of the same seeded stream): every
    rank's shard equals rows rank::world of the replicated table's initial values."""
    from recommendsystem_amd.embedding import SparseAdaGrad, SparseAdam, SparseTable
    for opt in (SparseAdam(), SparseAdaGrad()):
        full = SparseTable.initial_weight(10_007, 8, opt, 0.05, 9)
        for world in (1, 2, 3, 8):
            for rank in range(world):
                got = SparseTable.initial_shard(10_007, 8, opt, 0.05, 9, rank, world, chunk_rows=999)
                assert torch.equal(got, full[rank::world])
