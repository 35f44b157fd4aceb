"""The generic Trainer's HIP-graph path (Trainer.capture_pool / step_pool, what bench.py runs for
configs 3-5) trains exactly like its eager path: same parameters and tables after alternating
steps over a pool of batches (within fp32 sparse-sum tolerance: the pushes use float atomics),
and capture itself changes no state (its warm-up step is rolled back)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from _tol import assert_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _din(seed=2):
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd.workloads import DINPool
    d = DINPool(vocab=800, T=30, device=DEV, seed=seed)
    d.table.optimizer.learning_rate = 1e-2
    return d, Trainer(d, 1e-2, [d.table])


def _multi(seed=3):
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    from recommendsystem_amd.trainer import Trainer
    cfg = MultiHeadConfig(num_fields=40, vocab_per_field=300, lr_dense=1e-3, lr_sparse=1e-2)
    m = MultiHeadRanker(cfg, device=DEV, seed=seed)
    return m, Trainer(m, cfg.lr_dense, m.tables())


@pytest.mark.parametrize("which", ["din", "multi_head"])
def test_graph_pool_matches_eager(which):
    from recommendsystem_amd.workloads import din_batch, multi_head_batch
    rng = np.random.default_rng(90)
    if which == "din":
        mk = _din
        pool = [din_batch(rng, 64, 30, 800, DEV) for _ in range(2)]
    else:
        mk = _multi
        m0, _ = _multi()
        pool = [multi_head_batch(rng, 64, m0.cfg, DEV) for _ in range(2)]
    m_e, t_e = mk()
    m_g, t_g = mk()
    p0 = torch.cat([p.detach().reshape(-1) for p in m_g.parameters()]).clone()
    t_g.capture_pool(pool, warmup=1)
    p1 = torch.cat([p.detach().reshape(-1) for p in m_g.parameters()])
    assert torch.equal(p0, p1), "capture changed the parameters"
    losses_e, losses_g = [], []
    for i in range(4):
        losses_e.append(float(t_e.step(*pool[i % 2])))
        losses_g.append(float(t_g.step_pool(i)))
    torch.cuda.synchronize()
    assert_close(losses_g, losses_e, 1e-5, 1e-5, what="losses")
    pe = torch.cat([p.detach().reshape(-1) for p in m_e.parameters()]).cpu().numpy()
    pg = torch.cat([p.detach().reshape(-1) for p in m_g.parameters()]).cpu().numpy()
    assert_close(pg, pe, 2e-6, 1e-4, what="dense params")
    # tables: the sparse pushes sum with float atomics (order varies run to run) and Adam's
    # sign-like first steps pass an ill-conditioned row's rounding difference on at up to lr
    # scale: almost every entry matches closely, the rest within 2 lr
    for te, tg in zip(t_e.tables, t_g.tables):
        a, b = tg.weight.cpu().numpy(), te.weight.cpu().numpy()
        off = np.abs(a - b) > 2e-6 + 1e-4 * np.abs(b)
        assert off.mean() <= 1e-3, off.mean()
        assert_close(a, b, 2e-2, what="table")


def test_dropout_masks_fresh_per_replay():
    """Config 3's IL dropout under graph replay: one batch, one graph, lr 0 -- two replays give
    different losses (the device step counter offsets the seed, rs_set_seed_offset), and the
    same two losses as two eager steps (identical masks per step)."""
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    from recommendsystem_amd.trainer import Trainer
    from recommendsystem_amd.workloads import multi_head_batch
    cfg = MultiHeadConfig(num_fields=40, vocab_per_field=300, lr_dense=0.0, lr_sparse=0.0)
    batch = multi_head_batch(np.random.default_rng(4), 64, cfg, DEV)
    got = {}
    for mode in ("eager", "graph"):
        m = MultiHeadRanker(cfg, device=DEV, seed=5)
        t = Trainer(m, 0.0, m.tables())
        if mode == "graph":
            t.capture_pool([batch], warmup=1)
            got[mode] = [float(t.step_pool(i)) for i in range(3)]
        else:
            got[mode] = [float(t.step(*batch)) for _ in range(3)]
    assert len(set(got["graph"])) == 3, got
    assert_close(got["graph"], got["eager"], 1e-6, 1e-6, what="losses per step")
