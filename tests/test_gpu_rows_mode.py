"""The single-GPU AutoInt step's sparse Adam in rows mode (rs_partials_reduce_adam_rows: walk the
B x F looked-up rows, release each marked row's flag with an atomic exchange) against the flag
sweep (rs_partials_reduce_adam_scan): the same per-row update, so after captured steps every row was
updated exactly once per step it was touched in -- the tables agree to far below one Adam step
(lr 5e-5: a missed or doubled update differs by ~5e-5; the fused push's float atomics differ run
to run in the last bits), the Adam slots to fp32 rounding, and every flag is released.  Zipf-hot
rows appear hundreds of times per batch (many positions race for one flag)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(monkeypatch, maxn, pool_cpu, B):
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    monkeypatch.setenv("RS_SPARSE_ROWS_MAXN", str(maxn))
    cfg = AutoIntConfig()
    model = AutoInt(cfg, device=DEV, seed=0, max_batch=B)
    trainer = AutoIntTrainer(model, B)
    pool = [(i.to(DEV), l.to(DEV)) for i, l in pool_cpu]
    trainer.capture_pool(pool, warmup=0)
    for k in range(3):
        trainer.step_pool(k % len(pool))
    torch.cuda.synchronize()
    t = model.table
    return ([p.detach().clone() for p in model.parameters()],
            t.weight.clone(), t.m.clone(), t.v.clone(), t.flag.clone(), t.grad.abs().sum().item())


@pytest.mark.parametrize("B", [512, 1000])
def test_rows_mode_equals_sweep(monkeypatch, B):
    from recommendsystem_amd.autoint import AutoIntConfig
    cfg = AutoIntConfig()
    rng = np.random.default_rng(7)
    F, V = cfg.num_fields, cfg.vocab_per_field
    pool_cpu = []
    for _ in range(2):
        ids = np.minimum(rng.zipf(1.2, size=(B, F)) - 1, 10 * V).astype(np.int64)  # ids > V hash
        lab = (rng.uniform(size=(B, 1)) < 0.25).astype(np.float32)
        pool_cpu.append((torch.from_numpy(ids), torch.from_numpy(lab)))
    a = _run(monkeypatch, 10 ** 9, pool_cpu, B)   # rows mode
    b = _run(monkeypatch, 0, pool_cpu, B)         # flag sweep
    for x, y in zip(a[0], b[0]):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-6), "dense parameters differ"
    assert torch.allclose(a[1], b[1], rtol=0, atol=2e-6), \
        f"table: max diff {float((a[1] - b[1]).abs().max()):.3e} (one Adam step is ~5e-5)"
    touched_a = (a[3] != 0).any(1)
    touched_b = (b[3] != 0).any(1)
    assert torch.equal(touched_a, touched_b), "the sets of updated rows differ"
    assert torch.allclose(a[2], b[2], rtol=1e-3, atol=1e-9) and torch.allclose(a[3], b[3], rtol=1e-3, atol=1e-12)
    assert torch.equal(a[4], b[4]) and int((a[4] != -1).sum()) == 0, "flags not released"
    assert a[5] == 0.0 and b[5] == 0.0, "gradient rows not cleared"
