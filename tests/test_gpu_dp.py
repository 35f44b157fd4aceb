"""GPU, world size 2 on one device (gloo transport; RCCL on the 8-GPU node runs the same code):
the data-parallel AutoInt step (dist.exchange_packed: dense bucket + packed sparse records, two
all-gathers, rank-ordered merges and dense sum) after 3 steps over two alternating batches
(eager, and as one captured forward/backward graph per batch + one optimizer graph)

  * leaves bitwise-identical replicas (dense parameters and the embedding table), and
  * matches the CPU oracle's single-process train step on the union of the ranks' batches
    (same tolerances as test_gpu_parity::test_autoint_train_steps_match_oracle).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _tol import adam_close, assert_close, assert_grad_close

pytestmark = pytest.mark.gpu

B_LOCAL, WORLD, STEPS = 128, 2, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(max_batch, world):
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig
    cfg = AutoIntConfig(vocab_per_field=50, layer_num=3, lr_dense=1e-3, lr_sparse=1e-3)
    return cfg, AutoInt(cfg, device=torch.device("cuda", 0), seed=21, max_batch=max_batch,
                        world_size=world)


def _worker(rank, world, port, ids, labels, graph, out):
    """ids / labels: [NB, B_global, ...] global batches; step s trains on batch s % NB (rank r
    takes its slice).  graph: one captured forward/backward graph per batch + one optimizer
    graph, replayed alternately (capture_pool / step_pool)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from recommendsystem_amd.autoint import AutoIntTrainer
    cfg, model = _model(B_LOCAL, world)
    trn = AutoIntTrainer(model, B_LOCAL, process_group=dist.group.WORLD)
    assert trn.packed_dp
    sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
    pool = [(torch.from_numpy(i[sl]).cuda(), torch.from_numpy(l[sl]).cuda()) for i, l in zip(ids, labels)]
    if graph:
        trn.capture_pool(pool, warmup=1)  # the warm-up step is rolled back
        assert len(trn.pool_graphs) == len(pool)
        for s in range(STEPS):
            trn.step_pool(s)
    else:
        for s in range(STEPS):
            trn.step(*pool[s % len(pool)])
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).numpy()
    out[rank] = (params, model.table.weight.cpu().numpy(), float(trn.loss))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("graph", [False, True])
def test_dp_two_ranks_match_oracle(graph):
    from test_gpu_parity import _oracle_from_model
    B = B_LOCAL * WORLD
    cfg, model = _model(B, 1)
    rng = np.random.default_rng(21)
    NB = 2  # two different global batches, alternated
    ids = rng.integers(0, 10 * cfg.vocab_per_field, size=(NB, B, cfg.num_fields), dtype=np.int64)
    labels = (rng.uniform(size=(NB, B, 1)) < 0.25).astype(np.float32)
    ref, *_ = _oracle_from_model(model, cfg)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(WORLD, _free_port(), ids, labels, graph, out), nprocs=WORLD, join=True)
    p0, t0, l0 = out[0]
    p1, t1, l1 = out[1]
    assert np.array_equal(p0, p1), "dense replicas diverged"
    assert np.array_equal(t0, t1), "embedding-table replicas diverged"
    for st in range(STEPS):
        loss_ref = ref.step(torch.from_numpy(ids[st % NB]), torch.from_numpy(labels[st % NB]))
    # each rank's loss is its half-batch mean: their average is the global-batch loss
    assert abs(0.5 * (l0 + l1) - loss_ref) < 1e-5
    want = torch.cat([p.detach().reshape(-1) for p in ref.dense_list]).numpy()
    assert_close(p0.astype(np.float64), want, 2e-6, 1e-4, what="dense params after DP steps")
    assert_close(t0, ref.table.numpy(), 2e-6, 1e-4, what="table after DP steps")


def _worker_full(rank, world, port, out):
    """Config-2 size (B = 4096 per rank, 26 x 100k table), a 2-batch pool, graph-captured steps
    like bench.py (3 eager warm-up steps, then alternating batches)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    B = 4096
    cfg = AutoIntConfig()
    model = AutoInt(cfg, device=torch.device("cuda", 0), seed=0, max_batch=B, world_size=world)
    trn = AutoIntTrainer(model, B, process_group=dist.group.WORLD)
    rng = np.random.default_rng(2 + 1000 * rank)
    pool = []
    for k in range(2):  # a batch pool, as bench.py runs it (steps alternate between batches)
        z = np.minimum(rng.zipf(1.2, size=(B, cfg.num_fields)) - 1, cfg.vocab_per_field - 1)
        ids = torch.from_numpy(z.astype(np.int64)).cuda()
        g = torch.Generator().manual_seed(10 * rank + k)
        pool.append((ids, (torch.rand(B, 1, generator=g) < 0.25).float().cuda()))
    trn.capture_pool(pool, warmup=3)
    for i in range(2 * STEPS):
        trn.step_pool(i)
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).numpy()
    h = model.table.weight.double().sum(1).cpu().numpy()  # per-row checksum of the table
    # the last exchange's largest record count, read from the gathered buckets (the sync-free
    # exchange never reads it on the host itself)
    nmax = int(trn.dp_gathered_counts().max())
    out[rank] = (params, h, float(trn.loss), nmax)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_two_ranks_config2_size():
    """The full-size exchange (tens of thousands of records per rank): replicas stay identical."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_full, args=(WORLD, _free_port(), out), nprocs=WORLD, join=True)
    p0, h0, l0, n0 = out[0]
    p1, h1, l1, n1 = out[1]
    assert n0 == n1 > 10_000
    assert np.isfinite(l0) and np.isfinite(l1)
    assert np.array_equal(p0, p1) and np.array_equal(h0, h1)


# ------------------------------------------------------------------------------------------
# the generic Trainer (configs 3-5: trainer.py's all-reduce + list-mode sparse exchange)
# ------------------------------------------------------------------------------------------
B_DIN, T_DIN, V_DIN = 64, 20, 500


def _din_batches(world):
    from recommendsystem_amd.workloads import din_batch
    out = []
    for r in range(world):
        rng = np.random.default_rng(50 + r)
        out.append([a.cpu() for a in din_batch(rng, B_DIN, T_DIN, V_DIN, "cpu")])
    return out


def _union(batches):
    q = torch.cat([b[0] for b in batches])
    h = torch.cat([b[1] for b in batches])
    offs, base = [torch.zeros(1, dtype=torch.int32)], 0
    for b in batches:
        offs.append(b[2][1:] + base)
        base += int(b[2][-1])
    return q, h, torch.cat(offs), torch.cat([b[3] for b in batches])


def _din_trainer(pg):
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd.workloads import DINPool
    d = DINPool(vocab=V_DIN, T=T_DIN, device=torch.device("cuda", 0), seed=2)
    d.table.optimizer.learning_rate = 1e-2
    return d, Trainer(d, 1e-2, [d.table], process_group=pg)


def _worker_trainer(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d, trn = _din_trainer(dist.group.WORLD)
    grads = _record_grads(d, trn)
    batch = [a.cuda() for a in _din_batches(world)[rank]]
    for _ in range(STEPS):
        trn.step(*batch)
    torch.cuda.synchronize()
    d.table.check_overflow()
    params = torch.cat([p.detach().reshape(-1).cpu() for p in d.parameters()]).numpy()
    out[rank] = (params, d.table.weight.cpu().numpy(), grads)
    dist.barrier()
    dist.destroy_process_group()


def _record_grads(d, trn):
    """Per step: the exchanged dense gradient and the table gradient, both as the optimizers
    see them (times the 1/world scale)."""
    rec = []
    # the arena leaves alignment gaps between layers (trainer.ARENA_ALIGN): pack the gradient
    # in parameter order, as the parameters are compared
    base = trn.arena.data.data_ptr()
    spans = [((p.data_ptr() - base) // 4, p.numel()) for p in d.parameters()]

    def packed(g):
        return torch.cat([g[o:o + n] for o, n in spans])
    trn.on_dense_grad = lambda g, scale: rec.append(((packed(g) * scale).cpu().numpy(),
                                                     (d.table.grad * scale).cpu().numpy()))
    return rec


def _ill(got, want):
    """Entries whose two gradients differ by more than 0.1 % relative at any step: Adam's update
    is scale-free per entry, so such a difference reaches the parameter at ~lr x its size."""
    ill = np.zeros(np.asarray(want[0]).size, bool)
    for a, b in zip(got, want):
        a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
        ill |= np.abs(a - b) > 1e-3 * np.abs(b)
    return ill


def test_dp_generic_trainer_two_ranks():
    """2-rank DP of the generic Trainer (config-4 DIN harness, small vocab): bitwise-identical
    replicas, and the single-process Trainer on the union batch: the per-step dense and table
    gradients within the gradient tolerance, the parameters and table with the Adam
    ill-conditioning rule (tests/_tol.py::adam_close) -- the sparse sums use float atomics in a
    different order, and Adam (lr 1e-2 here) turns an entry's cancelled fp32 sum into a visible
    update difference."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_trainer, args=(WORLD, _free_port(), out), nprocs=WORLD, join=True)
    p0, t0, g0 = out[0]
    p1, t1, _ = out[1]
    assert np.array_equal(p0, p1), "dense replicas diverged"
    assert np.array_equal(t0, t1), "table replicas diverged"
    d, trn = _din_trainer(None)
    gu = _record_grads(d, trn)
    union = [a.cuda() for a in _union(_din_batches(WORLD))]
    for _ in range(STEPS):
        trn.step(*union)
    torch.cuda.synchronize()
    assert len(g0) == len(gu) == STEPS
    for s in range(STEPS):
        assert_grad_close(g0[s][0], gu[s][0], f"step {s + 1}: dense grad (DP vs union)")
        assert_grad_close(g0[s][1], gu[s][1], f"step {s + 1}: table grad (DP vs union)")
    want = torch.cat([p.detach().reshape(-1).cpu() for p in d.parameters()]).numpy()
    adam_close(p0, want, gu[-1][0], "dense params (DP vs union batch)",
               prev_ill=_ill([g[0] for g in g0], [g[0] for g in gu]))
    adam_close(t0, d.table.weight.cpu().numpy(), gu[-1][1], "table (DP vs union batch)",
               prev_ill=_ill([g[1] for g in g0], [g[1] for g in gu]))


def test_rccl_flat_all_gather_world1():
    """RCCL itself ('nccl' on ROCm) on this one-GPU box: a world-1 process group runs the
    packed exchange through all_gather_into_tensor (the path the 8-GPU node takes)."""
    from recommendsystem_amd import dist as rdist
    port = _free_port()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert rdist.uses_flat_all_gather()
        n_dense, ld, rs, cap = 10, 12, 5, 8
        send = torch.arange(ld, dtype=torch.float32, device="cuda")
        send.view(torch.int32)[n_dense] = 3  # record count
        recv = torch.zeros(ld, device="cuda")
        recs = torch.arange(cap * rs, dtype=torch.float32, device="cuda")
        recs_all = torch.zeros(cap * rs, device="cuda")
        nmax = rdist.exchange_packed(send, recv, n_dense, recs, recs_all, rs)
        torch.cuda.synchronize()
        assert nmax == 3
        assert torch.equal(recv, send)
        assert torch.equal(recs_all[:3 * rs], recs[:3 * rs])
    finally:
        dist.destroy_process_group()


_ONE_GRAPH_CHILD = r"""
import os, sys, traceback
sys.path.insert(0, sys.argv[1])
import numpy as np, torch, torch.distributed as dist
DEV = torch.device("cuda", 0)
os.environ["MASTER_ADDR"] = "127.0.0.1"
os.environ["MASTER_PORT"] = sys.argv[2]
dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
rc = 0
try:
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    B, NB, STEPS = 256, 2, 3
    cfg = AutoIntConfig(vocab_per_field=2000, layer_num=3, lr_dense=1e-3, lr_sparse=1e-3)
    rng = np.random.default_rng(5)
    # every (field, id) once per batch: each table row gets one push per step, so the float
    # atomics of the fused push add in a fixed order and eager == graph bitwise
    pool = []
    for k in range(NB):
        ids = np.stack([rng.permutation(cfg.vocab_per_field)[:B] for _ in range(cfg.num_fields)], 1)
        pool.append((torch.from_numpy(ids.astype(np.int64)).to(DEV),
                     torch.from_numpy((rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)).to(DEV)))
    res = {}
    for mode in ("eager", "one_graph", "split_graph"):
        if mode == "split_graph":
            os.environ["RS_DP_SPLIT_GRAPH"] = "1"
        model = AutoInt(cfg, device=DEV, seed=21, max_batch=B, world_size=1)
        trn = AutoIntTrainer(model, B, process_group=dist.group.WORLD, dp_world1=True)
        assert trn.packed_dp and trn.dp_sync_free
        assert trn.dp_one_graph == (mode != "split_graph")
        if mode == "eager":
            losses = [float(trn.step(*pool[s % NB])) for s in range(STEPS)]
        else:
            trn.capture_pool(pool, warmup=1)
            assert len(trn.pool_graphs) == NB
            assert (trn.graph_opt is None) == (mode == "one_graph")
            losses = [float(trn.step_pool(s)) for s in range(STEPS)]
        torch.cuda.synchronize()
        params = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
        res[mode] = (losses, params, model.table.weight.cpu().clone(), model.table.m.cpu().clone())
        os.environ.pop("RS_DP_SPLIT_GRAPH", None)
    e = res["eager"]
    for mode in ("one_graph", "split_graph"):
        g = res[mode]
        assert e[0] == g[0], (mode, e[0], g[0])
        for a, b in zip(e[1:], g[1:]):
            assert torch.equal(a, b), mode
    print("ONE-GRAPH-DP-OK", e[0], flush=True)
except Exception:
    traceback.print_exc()
    rc = 1
sys.stdout.flush()
sys.stderr.flush()
os._exit(rc)
"""


def test_dp_one_graph_rccl_world1():
    """The AutoInt data-parallel step as ONE captured graph per pool batch on RCCL (the merged
    all-gather inside the graph, thread_local capture): on a world-1 RCCL group (dp_world1: the
    DP code path -- exchange, rank-ordered merges, the fused dense sum + Adam) the replays equal
    the eager DP steps bitwise, and so does the two-graph form (RS_DP_SPLIT_GRAPH=1, what gloo
    runs).  Child process under a time limit."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ONE_GRAPH_CHILD, root, str(_free_port())],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and "ONE-GRAPH-DP-OK" in r.stdout, (r.stdout[-2000:] + r.stderr[-4000:])
