"""Shared tolerance helpers of the GPU parity tests (see tests/test_gpu_parity.py header)."""
from __future__ import annotations

import numpy as np


def to_np(t):
    return t.detach().double().cpu().numpy()


def assert_close(got, ref, atol, rtol=0.0, what=""):
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref)
    bound = atol + rtol * np.abs(ref)
    worst = np.max(err - bound) if err.size else -1
    assert worst <= 0, f"{what}: max|err|={err.max():.3e} (atol={atol}, rtol={rtol})"


def assert_grad_close(got, ref, what="", scale=2e-6):
    """Gradients: |err| <= 1e-4 |ref| + max(1e-4, scale max|ref|) (fp32 sums over many terms;
    scale grows with the length of the cancelling sums, e.g. 1e-5 for F > 64 fields)."""
    ref = np.asarray(ref, dtype=np.float64)
    assert_close(got, ref, max(1e-4, scale * float(np.abs(ref).max(initial=0.0))), 1e-4, what)


def adam_close(got, want, grad, what, atol=2e-6, rtol=1e-4, tiny=1e-6, max_frac=1e-3,
                grad_abs=None, cancel=1e-2, prev_ill=None):
    """Adam-updated parameters.  An entry is ill-conditioned when its gradient is ~0
    (|g| <= tiny * max|g|) or, given grad_abs = the sum of the |contributions| that make up g,
    when those contributions cancel to less than `cancel` of their magnitude (the fp32 sum then
    carries a relative error far above fp32 epsilon, and Adam's update m/(sqrt(v)+eps) passes
    it on at full scale).  Ill-conditioned entries may differ, but must be rare; all others
    must match.  prev_ill: entries ill-conditioned at an earlier step (their Adam moments carry
    the difference forward).  Returns this step's ill-conditioned mask (including prev_ill)."""
    got, want, grad = (np.asarray(a, dtype=np.float64).reshape(-1) for a in (got, want, grad))
    ill = np.abs(grad) <= tiny * max(float(np.abs(grad).max(initial=0.0)), 1e-30)
    if grad_abs is not None:
        ill |= np.abs(grad) < cancel * np.asarray(grad_abs, dtype=np.float64).reshape(-1)
    if prev_ill is not None:
        ill |= prev_ill
    bad = np.abs(got - want) > atol + rtol * np.abs(want)
    assert not np.any(bad & ~ill), (f"{what}: {int(np.sum(bad & ~ill))} mismatches, max|err| "
                                    f"{np.abs(got - want)[~ill].max():.3e}")
    assert np.sum(bad) <= max(2, max_frac * got.size), f"{what}: {int(np.sum(bad))} ill-conditioned"
    return ill
