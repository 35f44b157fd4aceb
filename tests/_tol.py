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
