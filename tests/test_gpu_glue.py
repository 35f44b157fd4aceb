"""GPU checks of the fused glue of the composed models against plain torch slicing / the
unfused ops (same forward values, same gradients):

* models.py _StaytimeFrontFn (staytime trunk fan-out: general / gate / query views of emb and
  the FFM, VideoDnn.py:11-25,45-47,57-77,99-105,127) against emb[:, :, 0:16], index_select and
  towers._FFMFn;
* din.py wide facts (rs_din_bwd_strided) against the sliced facts;
* towers.fused_loss against the per-output losses summed by torch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol, what):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    assert err <= tol * max(1.0, b.abs().max().item()), f"{what}: max|err| {err}"


def test_staytime_front_matches_views_and_ffm():
    from recommendsystem_amd.models import StaytimeConfig, StaytimeMTL, _StaytimeFrontFn
    from recommendsystem_amd.towers import _FFMFn
    torch.manual_seed(3)
    cfg = StaytimeConfig()
    m = StaytimeMTL(cfg, device=DEV, seed=5)
    B, F = 37, cfg.num_fields
    emb = (torch.rand(B, F, 32, device=DEV) - 0.5).requires_grad_(True)
    ffm = m.ffm
    nq = len(m.query_idx)
    w = [torch.randn(*t, device=DEV) for t in
         [(B, F, 16), (B, len(cfg.bias_fields) * 16)] + [(B, 16)] * nq +
         [(B, ffm.NU * ffm.NI * ffm.dim), (B, ffm.NU * 16)]]

    def loss(outs):
        return sum((o.reshape(B, -1) * g.reshape(B, -1)).sum() for o, g in zip(outs, w))

    outs = _StaytimeFrontFn.apply(emb, ffm.Wx, ffm.bx, ffm.Wy, ffm.by, m._front(F, 32))
    loss(outs).backward()
    g_emb = emb.grad.clone()
    g_par = [p.grad.clone() for p in (ffm.Wx, ffm.bx, ffm.Wy, ffm.by)]
    emb.grad = None
    for p in (ffm.Wx, ffm.bx, ffm.Wy, ffm.by):
        p.grad = None
    bias = torch.tensor(list(cfg.bias_fields), device=DEV)
    gen = emb[:, :, 0:16]
    y, mu = _FFMFn.apply(emb.reshape(B, -1), ffm.Wx, ffm.bx, ffm.Wy, ffm.by, ffm.cols, ffm.NU,
                         ffm.NI, ffm.dim, True)
    ref = [gen, emb.index_select(1, bias)[:, :, 16:32].reshape(B, -1)] + \
          [gen[:, q, :] for q in m.query_idx] + [y, mu]
    for a, b in zip(outs, ref):
        assert torch.equal(a.reshape(B, -1), b.reshape(B, -1))
    loss(ref).backward()
    _close(g_emb, emb.grad, 1e-6, "d emb")
    for a, p in zip(g_par, (ffm.Wx, ffm.bx, ffm.Wy, ffm.by)):
        _close(a, p.grad, 1e-6, "d ffm param")


def test_din_wide_facts_match_sliced():
    from recommendsystem_amd.din import StaytimeDIN
    torch.manual_seed(4)
    B, T = 29, 50
    d = StaytimeDIN(seed=2, device=DEV)
    d.build((1, T, 16), device=DEV)
    q = torch.randn(B, 16, device=DEV, requires_grad=True)
    facts = torch.randn(B, T, 32, device=DEV, requires_grad=True)
    mask = torch.rand(B, T, device=DEV) < 0.6
    mask[0] = False
    gw = torch.randn(B, 16, device=DEV)
    (d(q, facts, mask, wide=True) * gw).sum().backward()
    gq, gf = q.grad.clone(), facts.grad.clone()
    gW = d.W1.grad.clone()
    q.grad = facts.grad = None
    d.W1.grad = None
    (d(q, facts[:, :, 0:16], mask) * gw).sum().backward()
    assert torch.equal(gq, q.grad)
    assert torch.equal(gf, facts.grad)       # columns 16:32 exactly zero in both
    assert torch.equal(gW, d.W1.grad)


def test_fused_loss_matches_separate_terms():
    from recommendsystem_amd.towers import (bce_term, cross_entropy_sum, fused_loss, kd_mean_term,
                                            keras_bce, keras_bce_term)
    torch.manual_seed(5)
    M = 513
    p1 = torch.rand(M, 1, device=DEV).clamp(0.01, 0.99).requires_grad_(True)
    p2 = torch.rand(M, 1, device=DEV).clamp(0.01, 0.99).requires_grad_(True)
    s = torch.randn(M, 1, device=DEV, requires_grad=True)
    t = torch.randn(M, 1, device=DEV)
    y = (torch.rand(M, 1, device=DEV) < 0.3).float()
    sw = torch.where(torch.rand(M, device=DEV) < 0.1, 5.0, 1.0)
    L = fused_loss([bce_term(y, p1, 2.0, sample_weight=sw), keras_bce_term(y, p2),
                    kd_mean_term(s, t)], M)
    L.backward()
    g = [p1.grad.clone(), p2.grad.clone(), s.grad.clone()]
    p1.grad = p2.grad = s.grad = None
    ce = -(y * torch.log(p1 + 1e-6) + (1 - y) * torch.log(1 - p1 + 1e-6))
    ref = 2.0 * (ce.reshape(-1) * sw).mean() + keras_bce(y, p2) + ((s - t) ** 2).mean()
    ref.backward()
    _close(L, ref, 1e-6, "loss")
    for a, b, n in zip(g, [p1.grad, p2.grad, s.grad], ["d p1", "d p2", "d s"]):
        _close(a, b, 1e-5, n)
    assert cross_entropy_sum is not None
