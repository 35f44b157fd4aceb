"""Device training metrics (recommendsystem_amd/metrics.py, csrc/metrics.hip) against the numpy
restatement of tf.keras.metrics.AUC / binary accuracy / COPC / CTR (oracle/ctr_oracle.py):
accumulated over several batches, with and without sample weights, predictions placed exactly on
the fp32 thresholds and at the clip bounds (rank/ctr/base_model.py:183-190)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import ctr_oracle as npo

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("weighted", [False, True])
def test_ctr_metrics_match_oracle(weighted):
    from recommendsystem_amd.metrics import CtrMetrics
    rng = np.random.default_rng(3 + weighted)
    m = CtrMetrics(device=DEV)
    ps, ys, ws = [], [], []
    thr = (np.arange(1, 199) / 199.0).astype(np.float32)
    for k in range(3):
        B = 4096 if k < 2 else 1000
        y = (rng.uniform(size=B) < 0.25).astype(np.float32)
        p = np.clip(rng.beta(2, 5, size=B) + 0.2 * y, 1e-6, 1.0).astype(np.float32)
        p[:200] = rng.choice(thr, 200)            # exactly on thresholds (p > t is false there)
        p[200:210] = 1.0
        p[210:220] = 1e-6
        w = rng.uniform(0.5, 2.0, size=B).astype(np.float32) if weighted else None
        pt = torch.from_numpy(p).to(DEV).reshape(B, 1)
        yt = torch.from_numpy(y).to(DEV)
        m.update(pt, yt, torch.from_numpy(w).to(DEV) if weighted else None)
        ps.append(p); ys.append(y); ws.append(w)
    got = m.result()
    want = npo.ctr_metrics(np.concatenate(ps), np.concatenate(ys),
                           np.concatenate(ws) if weighted else None)
    for k in ("auc", "acc", "copc", "ctr", "pctr"):
        assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k])), (k, got[k], want[k])
    m.reset_states()
    assert m.result()["weight"] == 0.0


def test_ctr_metrics_strided_column():
    """A column of a wider output (the multi-task heads' [B, T] predictions)."""
    from recommendsystem_amd.metrics import CtrMetrics
    g = torch.Generator(device=DEV).manual_seed(4)
    P = torch.rand(512, 7, device=DEV, generator=g)
    Y = (torch.rand(512, 7, device=DEV, generator=g) < 0.3).float()
    m = CtrMetrics(device=DEV)
    m.update(P[:, 3:4], Y[:, 3:4])
    got = m.result()
    want = npo.ctr_metrics(P[:, 3].cpu().numpy(), Y[:, 3].cpu().numpy())
    assert abs(got["auc"] - want["auc"]) <= 1e-6 and abs(got["acc"] - want["acc"]) <= 1e-6


def test_autoint_trainer_metrics_match_oracle():
    """AutoIntTrainer(metrics=CtrMetrics()) accumulates AUC / acc / COPC over the steps' clipped
    predictions inside the captured step: equal to the oracle over the same (p, labels)."""
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    from recommendsystem_amd.metrics import CtrMetrics
    cfg = AutoIntConfig(vocab_per_field=1000)
    model = AutoInt(cfg, device=DEV, seed=1, max_batch=256)
    m = CtrMetrics(device=DEV)
    tr = AutoIntTrainer(model, 256, metrics=m)
    g = torch.Generator(device=DEV).manual_seed(5)
    ps, ys = [], []
    for k in range(3):
        ids = torch.randint(0, 1000, (256, 26), device=DEV, generator=g)
        lab = (torch.rand(256, 1, device=DEV, generator=g) < 0.25).float()
        tr.step(ids, lab)
        ps.append(tr.p.detach().cpu().numpy().copy())
        ys.append(lab.cpu().numpy())
    got = m.result()
    want = npo.ctr_metrics(np.concatenate(ps), np.concatenate(ys))
    for k in ("auc", "acc", "copc", "ctr"):
        assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k])), (k, got[k], want[k])


def test_autoint_trainer_metrics_per_task():
    """A two-task head (logits [2]) with one CtrMetrics per task: task t accumulates column t of
    p and labels (a single CtrMetrics for T = 2 is refused at construction)."""
    import pytest
    from recommendsystem_amd.autoint import AutoInt, AutoIntConfig, AutoIntTrainer
    from recommendsystem_amd.metrics import CtrMetrics
    cfg = AutoIntConfig(vocab_per_field=1000, logits_hidden=(2,))
    model = AutoInt(cfg, device=DEV, seed=1, max_batch=128)
    with pytest.raises(ValueError):
        AutoIntTrainer(model, 128, metrics=CtrMetrics(device=DEV))
    ms = [CtrMetrics(device=DEV), CtrMetrics(device=DEV)]
    tr = AutoIntTrainer(model, 128, metrics=ms)
    g = torch.Generator(device=DEV).manual_seed(6)
    ps, ys = [], []
    for _ in range(2):
        ids = torch.randint(0, 1000, (128, 26), device=DEV, generator=g)
        lab = (torch.rand(128, 2, device=DEV, generator=g) < 0.3).float()
        tr.step(ids, lab)
        ps.append(tr.p.detach().cpu().numpy().copy())
        ys.append(lab.cpu().numpy())
    P, Y = np.concatenate(ps), np.concatenate(ys)
    for t in range(2):
        got = ms[t].result()
        want = npo.ctr_metrics(P[:, t:t + 1], Y[:, t:t + 1])
        for k in ("auc", "acc", "copc", "ctr"):
            assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k])), (t, k, got[k], want[k])
