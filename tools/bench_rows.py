"""Per-row kernel measurements for the §8 rows beyond the headline bench (one JSON line per
kernel): average launch time (HIP events on the launch stream), algorithmic bytes (and flops)
per launch, and the achieved fraction of the HBM roofline (8 TB/s, MI355X_MICROARCH.md).

    python tools/bench_rows.py [--reps 50]

Workloads (SURVEY §8d synthetic configs, per GPU):
  din_fwd / din_bwd        config 4: B=4096, T=100, H=16, keys = values (one lookup), lengths
                           U{1..100}
  staytime_din_fwd / _bwd  config 5: B=2048 per GPU (16384 / DP 8), T=50, H=16, facts are the
                           [:, :, 0:16] slice of a 32-wide sequence lookup, mask from lengths
  seq_lookup               config 4 history lookup: 4096 x 100 ids into a 1M x 16 table
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402

HBM_GBS = 8000.0


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def report(name, t, bytes_, flops=None, **extra):
    d = {"kernel": name, "us": round(t * 1e6, 2), "alg_bytes": int(bytes_),
         "GBps": round(bytes_ / t / 1e9, 1), "hbm_frac": round(bytes_ / t / 1e9 / HBM_GBS, 4)}
    if flops:
        d["TFLOPs"] = round(flops / t / 1e12, 3)
    d.update(extra)
    print(json.dumps(d), flush=True)


def din_case(variant, B, T, reps, strided):
    lib = _lib.load()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(variant)
    H = 16
    q = (torch.rand(B, H, device=dev, generator=g) - 0.5)
    if strided:
        kfull = (torch.rand(B, T, 2 * H, device=dev, generator=g) - 0.5)
        k = kfull[:, :, :H]
    else:
        k = (torch.rand(B, T, H, device=dev, generator=g) - 0.5)
    lens = torch.randint(1, T + 1, (B,), device=dev, generator=g, dtype=torch.int32)
    mask = None
    if variant == 1:
        mask = (torch.arange(T, device=dev)[None, :] < lens[:, None]).to(torch.uint8)
    nb = 3 if variant == 0 else 4
    W1 = (torch.rand(nb * H, 16, device=dev, generator=g) - 0.5) * 0.5
    b1 = torch.zeros(16, device=dev)
    W2 = (torch.rand(16, 1, device=dev, generator=g) - 0.5)
    b2 = torch.full((1,), 0.05, device=dev)
    out = torch.empty(B, H, device=dev)
    probs = torch.empty(B, T, device=dev) if variant == 1 else None
    dout = torch.randn(B, H, device=dev, generator=g)
    dq = torch.empty(B, H, device=dev)
    dk = torch.empty(B, T, H, device=dev)
    np_ = int(lib.rs_din_param_count(variant, H))
    dpar = torch.empty(np_, device=dev)
    wsn = int(lib.rs_din_bwd_workspace_floats(variant, B, T, H))
    ws = torch.empty(wsn, device=dev)
    s = stream_handle()
    lens_p = ptr(lens) if variant == 0 else None
    m_p = ptr(mask)
    fwd = lambda: call("rs_din_fwd", s, variant, ptr(q), H, ptr(k), k.stride(0), k.stride(1), ptr(k),  # noqa: E731
                       k.stride(0), k.stride(1), B, T, H, lens_p, m_p, T, ptr(W1), ptr(b1), ptr(W2),
                       ptr(b2), ptr(out), H, ptr(probs))
    bwd = lambda: call("rs_din_bwd", s, variant, ptr(q), H, ptr(k), k.stride(0), k.stride(1), ptr(k),  # noqa: E731
                       k.stride(0), k.stride(1), B, T, H, lens_p, m_p, T, ptr(W1), ptr(b1), ptr(W2),
                       ptr(b2), ptr(probs), ptr(dout), H, ptr(dq), H, ptr(dk), ptr(dk), ptr(dpar), 0,
                       ptr(ws), wsn)
    tf = timed(fwd, reps)
    tb = timed(bwd, reps)
    row = T * H * 4
    side = 4 if variant == 0 else T  # lengths int32 | mask bytes
    fwd_bytes = B * (H * 4 + row + side + H * 4 + (T * 4 if variant == 1 else 0))
    bwd_bytes = B * (H * 4 + row + side + H * 4 + H * 4 + row + (T * 4 if variant == 1 else 0))
    name = "din" if variant == 0 else "staytime_din"
    fl_f = B * T * (2 * H * 16 + 2 * 16) + B * T * H * 2
    report(f"{name}_fwd", tf, fwd_bytes, fl_f, B=B, T=T, strided=strided)
    report(f"{name}_bwd", tb, bwd_bytes, 3 * fl_f, B=B, T=T, strided=strided,
           partial_bytes=wsn * 4)


def seq_case(B, T, vocab, reps):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    dim = 16
    table = torch.rand(vocab, dim, device=dev, generator=g)
    ids = torch.randint(0, vocab, (B * T,), device=dev, generator=g, dtype=torch.int64)
    offs = torch.arange(0, B * T + 1, T, device=dev, dtype=torch.int32)
    out = torch.empty(B, T, dim, device=dev)
    mask = torch.empty(B, T, device=dev, dtype=torch.uint8)
    rows = torch.empty(B * T, device=dev, dtype=torch.int32)
    s = stream_handle()
    fn = lambda: call("rs_sequence_lookup_fwd", s, ptr(ids), ptr(offs), B, T, 0, vocab, 0,  # noqa: E731
                      ptr(table), dim, ptr(out), T * dim, dim, ptr(mask), T, None, ptr(rows))
    t = timed(fn, reps)
    report("seq_lookup", t, B * T * (8 + 64 + 64 + 1 + 4) + B * 8, None, B=B, T=T, vocab=vocab)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    din_case(0, 4096, 100, a.reps, False)
    din_case(1, 2048, 50, a.reps, True)
    din_case(1, 16384, 50, a.reps, True)
    seq_case(4096, 100, 1_000_000, a.reps)


if __name__ == "__main__":
    main()
