"""staytime input parsing: ``parse_input_func`` of ``staytime/parse.py:16-71`` on an
already-decoded batch, with the label construction on the GPU (``rs_staytime_labels``).

The reference parses serialized ``tf.Example`` protos; here the TFRecord framing and the
``tf.train.Example`` decode happen in ``data.py`` (``dataset_reader`` / ``decode_batch``), so a batch
arrives at this function as a dict of decoded columns:

    {"extra_info": [str] * B (default "label", parse.py:18),
     "video_duration": int64 [B], "watch_duration": int64 [B],
     <slot>: int64 ids — [B, k] dense or (values, row_splits) ragged, parse.py:22-23}

and the function returns the reference's triple ``(feature_dict, y, sample_weight)`` with the same
keys: ``watch_duration`` and ``extra_info`` popped, ``example_id`` = extra_info (parse.py:26-28),
``y`` keyed ``<prefix>_staytime`` ([B, 401] = 400 soft-label bins ++ clipped seconds),
``<prefix>_shortplay`` and ``<prefix>_longplay`` ([B, 1]; fp32 0/1 where the reference keeps
int64 — the losses consume fp32), ``sample_weight`` [B, 1].  The only host work is the
extra_info regex (string matching), reduced to one byte per sample before the launch.
"""
from __future__ import annotations

import re
from typing import Sequence

import numpy as np
import torch

from ._lib import call, ptr, stream_handle
from .models import STAYTIME_BINS

MODEL_PREFIX = "video_id_rank_staytime_mtl_ppnet_v7"                      # parse.py:67-69
LANDING_PATTERN = re.compile(r".*video_homepage_landing.*")             # parse.py:64
SIGMA, LEFT, RIGHT = 4.0, -19.0, 180.5                                  # parse.py:55-58

_BINS_CACHE: dict[torch.device, torch.Tensor] = {}


def _bins(device: torch.device, bins: Sequence[float] | None) -> torch.Tensor:
    if bins is not None:
        return torch.as_tensor(bins, dtype=torch.float32, device=device).contiguous()
    if device not in _BINS_CACHE:
        _BINS_CACHE[device] = torch.tensor(STAYTIME_BINS, dtype=torch.float32, device=device)
    return _BINS_CACHE[device]


def staytime_labels(watch_ms: torch.Tensor, landing: torch.Tensor | None = None,
                    bins: Sequence[float] | None = None, sigma: float = SIGMA,
                    left: float = LEFT, right: float = RIGHT):
    """Device labels of parse.py:30-64 from int64 watch times in ms [B] (and an optional uint8
    landing flag [B]) -> (staytime [B, nbins + 1], short [B, 1], long [B, 1], weight [B, 1])."""
    if watch_ms.device.type != "cuda":
        raise ValueError("staytime_labels: watch_ms must be a device tensor (no CPU path)")
    watch_ms = watch_ms.reshape(-1).to(torch.int64).contiguous()
    dev = watch_ms.device
    B = watch_ms.numel()
    b = _bins(dev, bins)
    nb = b.numel()
    if landing is not None:
        landing = landing.reshape(-1).to(device=dev, dtype=torch.uint8).contiguous()
        if landing.numel() != B:
            raise ValueError(f"landing has {landing.numel()} entries for {B} samples")
    stay = torch.empty(B, nb + 1, device=dev)
    short, long_, sw = (torch.empty(B, 1, device=dev) for _ in range(3))
    call("rs_staytime_labels", stream_handle(), ptr(watch_ms), ptr(landing), B, ptr(b), nb,
         sigma, left, right, ptr(stay), nb + 1, ptr(short), ptr(long_), ptr(sw))
    return stay, short, long_, sw


def landing_flags(extra_info: Sequence[str | bytes]) -> np.ndarray:
    """tf.strings.regex_full_match(extra_info, ".*video_homepage_landing.*") (parse.py:64)."""
    out = np.zeros(len(extra_info), dtype=np.uint8)
    for i, s in enumerate(extra_info):
        if isinstance(s, bytes):
            s = s.decode("utf-8", "replace")
        out[i] = LANDING_PATTERN.fullmatch(s) is not None
    return out


def _to_device(v, device):
    """host column -> device int64 (pinned host tensors copy asynchronously)."""
    if isinstance(v, tuple):          # ragged (values, row_splits)
        return tuple(_to_device(a, device) for a in v)
    if isinstance(v, torch.Tensor):
        return v.to(device=device, dtype=torch.int64, non_blocking=v.is_pinned())
    return torch.as_tensor(np.asarray(v), dtype=torch.int64).to(device)


def parse_input_func(example: dict, device: str | torch.device = "cuda",
                     prefix: str = MODEL_PREFIX):
    """staytime/parse.py:16-71 on a decoded batch -> (feature_dict, y, sample_weight)."""
    ex = dict(example)
    if "watch_duration" not in ex or "video_duration" not in ex:
        raise KeyError("parse_input_func: watch_duration and video_duration are required "
                       "(FixedLenFeature without default, parse.py:19-20)")
    wt = ex.pop("watch_duration")
    wt = wt.to(torch.int64) if isinstance(wt, torch.Tensor) else torch.as_tensor(np.asarray(wt), dtype=torch.int64)
    B = wt.numel()
    extra_info = list(ex.pop("extra_info", ["label"] * B))              # parse.py:18 default
    if len(extra_info) != B:
        raise ValueError(f"extra_info has {len(extra_info)} entries for {B} samples")
    landing = torch.from_numpy(landing_flags(extra_info))
    features = {k: _to_device(v, device) for k, v in ex.items()}
    features["example_id"] = extra_info                                 # parse.py:27
    stay, short, long_, sw = staytime_labels(wt.to(device, non_blocking=wt.is_pinned()), landing)
    y = {f"{prefix}_staytime": stay, f"{prefix}_shortplay": short,
         f"{prefix}_longplay": long_}
    return features, y, sw
