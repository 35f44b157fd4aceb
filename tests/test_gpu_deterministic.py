"""The deterministic sparse push (rs_sparse_grad_accumulate_sorted: sort + segmented sum,
SURVEY §7.2) and the AutoInt trainer's deterministic mode: the same sums as the fp64 oracle, the
same touched-row sets as the atomic push, and bitwise-identical results run to run."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo
from _tol import assert_close, assert_grad_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _push(table_rows, dim, rows, offsets, B, F, dout, combiner, deterministic, mode="list"):
    from recommendsystem_amd.embedding import SparseTable
    t = SparseTable(table_rows, dim, device=DEV)
    t.mode = mode
    t.deterministic = deterministic
    t.accumulate(rows, offsets, B, F, dout, F * dim, dim, combiner)
    torch.cuda.synchronize()
    return t


@pytest.mark.parametrize("multi_hot", [False, True])
@pytest.mark.parametrize("mode", ["list", "scan"])
def test_sorted_push_matches_oracle_and_atomic(multi_hot, mode):
    rng = np.random.default_rng(70)
    B, F, dim, R = 300, 7, 16, 500
    if multi_hot:
        lens = rng.integers(0, 4, size=B * F)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        comb, cname = 1, "mean"
    else:
        offs, comb, cname = None, 0, "sum"
    n = int(offs[-1]) if multi_hot else B * F
    # Zipf-like collisions plus invalid (-1) ids
    r = np.minimum(rng.zipf(1.3, size=n) - 1, R - 1).astype(np.int32)
    r[rng.uniform(size=n) < 0.05] = -1
    dout = rng.standard_normal((B, F * dim)).astype(np.float32)
    rows_d = torch.from_numpy(r).to(DEV)
    offs_d = torch.from_numpy(offs).to(DEV) if multi_hot else None
    dout_d = torch.from_numpy(dout).to(DEV)
    det = _push(R, dim, rows_d, offs_d, B, F, dout_d, comb, True, mode)
    atm = _push(R, dim, rows_d, offs_d, B, F, dout_d, comb, False, mode)
    want = npo.sparse_grad_sum(r, offs, B, F, dout.astype(np.float64), cname)
    keys = np.array(sorted(k for k in want if k >= 0))
    got = det.grad.cpu().numpy()
    assert_grad_close(got[keys], np.stack([want[k] for k in keys]), "sorted push")
    untouched = np.setdiff1d(np.arange(R), keys)
    assert not np.any(got[untouched]), "rows nobody pushed were written"
    assert_close(got, atm.grad.cpu().numpy(), 1e-5, 1e-5, what="sorted vs atomic push")
    if mode == "list":
        for t in (det, atm):
            cnt = int(t.n_touched[0])
            assert cnt == keys.size
            assert np.array_equal(np.sort(t.touched[:cnt].cpu().numpy()), keys)
    flag_det, flag_atm = det.flag.cpu().numpy(), atm.flag.cpu().numpy()
    assert np.array_equal(flag_det, flag_atm)
    assert set(np.nonzero(flag_det == -2)[0].tolist()) == set(keys.tolist())
    # bitwise reproducible: a second deterministic push of the same inputs
    det2 = _push(R, dim, rows_d, offs_d, B, F, dout_d, comb, True, mode)
    assert torch.equal(det.grad, det2.grad)


def test_sorted_push_sequence_layout_and_bounds():
    """Sequence pushes (offsets NULL, [B, T] slots with -1 padding) and ids outside the table."""
    rng = np.random.default_rng(71)
    B, T, dim, R = 64, 50, 32, 1000
    r = rng.integers(0, R + 20, size=B * T).astype(np.int32)  # some rows >= R: push nothing
    r[rng.uniform(size=B * T) < 0.3] = -1
    dout = rng.standard_normal((B, T * dim)).astype(np.float32)
    t = _push(R, dim, torch.from_numpy(r).to(DEV), None, B, T, torch.from_numpy(dout).to(DEV), 0, True)
    rv = np.where(r >= R, -1, r)
    want = npo.sparse_grad_sum(rv, None, B, T, dout.astype(np.float64), "sum")
    keys = np.array(sorted(k for k in want if k >= 0))
    assert_grad_close(t.grad.cpu().numpy()[keys], np.stack([want[k] for k in keys]), "sequence push")
    assert int(t.n_touched[0]) == keys.size


def test_autoint_deterministic_trainer_is_bitwise_reproducible():
    """Two trainers from the same init over the same Zipf batches (captured pool graphs): every
    parameter and every table row bitwise equal after 3 steps; and close to the atomic trainer."""
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    B = 1024
    cfg = AutoIntConfig(vocab_per_field=5000, lr_dense=1e-3, lr_sparse=1e-3)
    rng = np.random.default_rng(72)
    pool = [(torch.from_numpy(np.minimum(rng.zipf(1.2, size=(B, 26)) - 1, 4999).astype(np.int64)).to(DEV),
             torch.from_numpy((rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)).to(DEV))
            for _ in range(2)]
    states = []
    for det in (True, True, False):
        model = AutoInt(cfg, device=DEV, seed=1, max_batch=B)
        tr_ = AutoIntTrainer(model, B, deterministic=det)
        tr_.capture_pool(pool, warmup=1)
        for i in range(3):
            tr_.step_pool(i)
        torch.cuda.synchronize()
        states.append((torch.cat([p.detach().reshape(-1) for p in model.parameters()]).clone(),
                       model.table.weight.clone()))
    (p1, t1), (p2, t2), (p3, t3) = states
    assert torch.equal(p1, p2) and torch.equal(t1, t2), "deterministic trainer not reproducible"
    # the atomic trainer differs only by summation order (Adam can magnify it on ill-conditioned
    # entries: compare loosely, most entries tightly)
    off = (p1 - p3).abs() > 2e-6 + 1e-4 * p3.abs()
    assert float(off.float().mean()) < 1e-2
    offt = (t1 - t3).abs() > 2e-6 + 1e-4 * t3.abs()
    assert float(offt.float().mean()) < 1e-3
