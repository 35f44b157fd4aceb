"""The configs 3-5 CPU train-step ports bench.py times as cpu_baseline (oracle/torch_ref.py
MultiHeadCPU / DINPoolCPU, oracle/model_oracles.py StaytimeRoughRankCPU): they run on CPU-built
models, train (the loss falls on a repeated batch), and the config-5 port's sparse AdaGrad update
of the shared table matches ctr_oracle.adagrad_sparse on the fp64 oracle's summed row gradients."""
import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from oracle import torch_ref as tr
from oracle.model_oracles import StaytimeRoughRankCPU, dssm_oracle, staytime_oracle
from recommendsystem_amd import workloads as W


def _staytime_batch_cpu(rng, B, j):
    """workloads.staytime_batch with host labels (workloads.staytime_labels)."""
    st, rr = j.st_cfg, j.rr_cfg
    t = torch.from_numpy
    st_ids = W.zipf_ids(rng, (B, st.num_fields), 1 << 40, 1.2)
    si, so = [], []
    for _ in range(st.num_seq):
        lens = rng.integers(0, st.seq_len + 1, size=B)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        si.append(t(W.zipf_ids(rng, (int(offs[-1]),), 1 << 40, 1.2)))
        so.append(t(offs))
    rr_ids = W.zipf_ids(rng, (B, rr.user_fields + rr.item_fields), 1 << 40, 1.2)
    stay, short, long_, sw = [t(np.ascontiguousarray(a)) for a in W.staytime_labels(rng, B)]
    click = t((rng.uniform(size=(B, 1)) < 0.1).astype(np.float32))
    mask = t((rng.uniform(size=(B, 1)) < 0.5).astype(np.float32))
    return (t(st_ids), si, so, t(rr_ids), stay, short, long_, sw, click, mask)


def _falls(ref, batch, steps=6):
    losses = [ref.step(*batch) for _ in range(steps)]
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses
    return losses


def test_multi_head_cpu_port_trains():
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    rng = np.random.default_rng(1)
    cfg = MultiHeadConfig()
    model = MultiHeadRanker(cfg, device="cpu", seed=0)
    ref = tr.MultiHeadCPU(model, lr_dense=1e-3, lr_sparse=1e-2)
    _falls(ref, ref.prepare(*W.multi_head_batch(rng, 32, cfg, "cpu")))


def test_din_cpu_port_trains():
    rng = np.random.default_rng(2)
    model = W.DINPool(vocab=5000, device="cpu", seed=0)
    ref = tr.DINPoolCPU(model, lr_dense=1e-3, lr_sparse=1e-2)
    _falls(ref, ref.prepare(*W.din_batch(rng, 64, model.T, 5000, "cpu")))


def test_staytime_cpu_port_matches_oracle_and_adagrad():
    rng = np.random.default_rng(3)
    j = W.StaytimeRoughRank(rows=4096, device="cpu", seed=3)
    B = 16
    batch = _staytime_batch_cpu(rng, B, j)
    ref = StaytimeRoughRankCPU(j)
    prep = ref.prepare(batch)
    rows_f, seq, rows_r = prep[0], prep[1], prep[2]
    cfg, rcfg = j.st_cfg, j.rr_cfg
    F, nrr = cfg.num_fields, rcfg.user_fields + rcfg.item_fields
    W0 = ref.table.numpy().astype(np.float64)
    g20 = ref.g2sum.numpy().astype(np.float64)
    # fp64 oracle on the same rows: loss and every touched row's summed gradient
    e64 = torch.tensor(W0[rows_f.numpy()].reshape(B, F, -1), requires_grad=True)
    s64, mk = [], []
    for r_, m_ in seq:
        g = W0[r_.clamp(min=0).numpy()] * (r_.numpy() >= 0)[..., None]
        s64.append(torch.tensor(g, requires_grad=True))
        mk.append(m_)
    r64 = torch.tensor(W0[rows_r.numpy()][:, 0:16].reshape(B, nrr, 16), requires_grad=True)
    stay, short, long_, sw, click, mask = batch[4:]
    o = staytime_oracle(j.staytime, cfg, e64, s64, mk, stay, short, long_, sw)
    d = dssm_oracle(j.dssm, r64, mask, click)
    loss64 = o["loss"] + d["loss"]
    loss64.backward()
    g: dict[int, np.ndarray] = {}

    def add(rows, grads):
        for r, gg in zip(rows.tolist(), grads):
            if r >= 0:
                g[r] = g[r] + gg if r in g else gg.copy()

    add(rows_f.numpy(), e64.grad.numpy().reshape(-1, 32))
    for (r_, _), s in zip(seq, s64):
        add(r_.numpy().reshape(-1), s.grad.numpy().reshape(-1, 32))
    rg = np.zeros((B * nrr, 32))
    rg[:, :16] = r64.grad.numpy().reshape(-1, 16)
    add(rows_r.numpy(), rg)

    loss32 = ref.step(*prep)
    loss64 = float(loss64.detach())
    assert abs(loss32 - loss64) <= 1e-4 * max(1.0, abs(loss64))
    keys = np.array(sorted(g), dtype=np.int64)
    gs = np.stack([g[k] for k in keys])
    w_ref, g2_ref = npo.adagrad_sparse(W0[keys], gs, g20[keys], ref.lr_sparse)
    np.testing.assert_allclose(ref.table.numpy()[keys], w_ref, rtol=0, atol=2e-5)
    # g2sum accumulates squared fp32 gradients (hot rows sum many occurrences): relative 1e-2
    np.testing.assert_allclose(ref.g2sum.numpy()[keys], g2_ref, rtol=1e-2, atol=1e-6)
    untouched = np.setdiff1d(np.arange(4096), keys)
    assert np.array_equal(ref.table.numpy()[untouched], W0[untouched].astype(np.float32))
    # and it keeps training
    _falls(ref, prep, steps=4)


@pytest.mark.parametrize("n", [0])
def test_staytime_cpu_port_empty_sequences(n):
    """All history sequences empty (every row -1, mask False): the port still steps."""
    rng = np.random.default_rng(4)
    j = W.StaytimeRoughRank(rows=1024, device="cpu", seed=5)
    b = list(_staytime_batch_cpu(rng, 8, j))
    b[1] = [torch.zeros(n, dtype=torch.int64) for _ in b[1]]
    b[2] = [torch.zeros(9, dtype=torch.int32) for _ in b[2]]
    ref = StaytimeRoughRankCPU(j)
    prep = ref.prepare(tuple(b))
    assert all(bool((r_ < 0).all()) and not bool(m_.any()) for r_, m_ in prep[1])
    assert np.isfinite(ref.step(*prep))
