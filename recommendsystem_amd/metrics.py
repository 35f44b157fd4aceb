"""Training metrics of the reference's model.compile calls, on the device:
Keras 'acc' / BinaryAccuracy(), tf.keras.metrics.AUC() (200 thresholds, ROC, interpolation) and
tensornet's tn.metric.COPC() / CTR() -- rank/ctr/base_model.py:183-190 (metrics and
weighted_metrics), rough_rank/model.py:215-219, rank/multi_head/model.py:55,
staytime/model.py:81-82.

``CtrMetrics.update(p, y[, w])`` enqueues one accumulation kernel (no host read; safe inside a
captured HIP graph); ``result()`` reads the totals back (call it between steps, like Keras'
per-epoch / logging read-out); ``reset_states()`` zeroes them.  Kernels: csrc/metrics.hip.
The totals are fp64 atomics: counts are exact, but WEIGHTED sums (non-integer w) depend on the
order the blocks arrive in, so they can differ in the last bits from run to run.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr, stream_handle

NAMES = ("auc", "acc", "copc", "ctr", "pctr", "weight")


class CtrMetrics:
    def __init__(self, num_thresholds: int = 200, device=None):
        n = int(_lib.load().rs_ctr_metrics_state_doubles(num_thresholds))
        if n < 0:
            raise ValueError(f"num_thresholds must be in [3, 1024], got {num_thresholds}")
        self.num_thresholds = num_thresholds
        self.state = torch.zeros(n, device=device or "cuda", dtype=torch.float64)
        self.out = torch.zeros(len(NAMES), device=self.state.device, dtype=torch.float32)

    def update(self, p: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None = None) -> None:
        """p, y (and w): one column each ([B] or [B, 1]; strided columns of a wider output are
        fine: the row stride is passed through)."""
        _lib.require_device(p, y, w)
        B = p.shape[0]
        if y.shape[0] != B or (w is not None and w.shape[0] != B):
            raise ValueError("predictions, labels and weights need the same batch size")

        def col(t):
            if t.dim() == 1:
                return t.stride(0)
            if t.dim() == 2 and t.shape[1] == 1:
                return t.stride(0)
            raise ValueError("metric inputs are one column ([B] or [B, 1])")

        for t in (p, y) + ((w,) if w is not None else ()):
            if t.dtype != torch.float32:
                raise ValueError("metric inputs must be float32")
        call("rs_ctr_metrics_accumulate", stream_handle(), ptr(p), col(p), ptr(y), col(y),
             ptr(w), col(w) if w is not None else 1, B, self.num_thresholds, ptr(self.state))

    def result(self) -> dict:
        call("rs_ctr_metrics_result", stream_handle(), ptr(self.state), self.num_thresholds,
             ptr(self.out))
        vals = self.out.tolist()
        return dict(zip(NAMES, vals))

    def reset_states(self) -> None:
        self.state.zero_()
