"""Time the sparse push (rs_sparse_grad_accumulate) at the workload shapes, each launch alone with
the sparse optimizer run in between (flags / gradient rows reset as in a training step):

  c3      config 3: B = 4096 x 200 fields, multi-hot U{1..3} (mean), Zipf(1.2) over 265 k per
          field (disjoint row ranges), dim 8, list mode
  c4_hist config 4: the DIN history, B = 1024 x T = 100 positions over one 1 M x 16 table,
          Zipf(1.1), lengths U{1..100} (padded positions row -1), list mode
  c4_q    config 4: the query push, B = 1024 single-hot
  c2      config 2: B = 4096 x 26 single-hot fields over 26 x 100 k, dim 16, scan mode
  c3_scan config 3's push in scan mode (no claims)
  c5      config 5: B = 2048 x 91 single-hot hashed fields over one 10 M x 32 table, list mode

python tools/push_bench.py [--reps N] [--only c3,c4_hist]  -> one JSON line
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from recommendsystem_amd import _lib
from recommendsystem_amd.embedding import SparseAdam, SparseTable


def zipf(rng, shape, vocab, a):
    return np.minimum(rng.zipf(a, size=shape) - 1, vocab - 1)


def case_c3(rng, dev):
    B, F, V, D = 4096, 200, 265_000, 8
    lens = rng.integers(1, 4, size=B * F)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    seg = np.repeat(np.arange(B * F), lens)
    rows = (seg % F) * V + zipf(rng, (int(offs[-1]),), V, 1.2)
    t = SparseTable(F * V, D, SparseAdam(1e-3), device=dev, max_touched=B * F * 3)
    dout = torch.randn(B, F * D, device=dev)
    r = torch.from_numpy(rows.astype(np.int32)).to(dev)
    o = torch.from_numpy(offs).to(dev)
    return t, lambda: t.accumulate(r, o, B, F, dout, F * D, D, 1), rows


def case_c4_hist(rng, dev):
    B, T, V, D = 1024, 100, 1_000_000, 16
    lens = rng.integers(1, T + 1, size=B)
    lens[0] = T
    ids = zipf(rng, (B, T), V, 1.1)
    ids[np.arange(T)[None, :] >= lens[:, None]] = -1
    t = SparseTable(V, D, SparseAdam(1e-3), device=dev, max_touched=B * T + B)
    dout = torch.randn(B, T, D, device=dev)
    r = torch.from_numpy(ids.astype(np.int32).reshape(-1)).to(dev)
    return t, lambda: t.accumulate(r, None, B, T, dout, T * D, D, 0), ids[ids >= 0]


def case_c4_q(rng, dev):
    B, V, D = 1024, 1_000_000, 16
    ids = zipf(rng, (B,), V, 1.1)
    t = SparseTable(V, D, SparseAdam(1e-3), device=dev, max_touched=B * 101)
    dout = torch.randn(B, D, device=dev)
    r = torch.from_numpy(ids.astype(np.int32)).to(dev)
    return t, lambda: t.accumulate(r, None, B, 1, dout, D, D, 0), ids


def case_c2(rng, dev):
    B, F, V, D = 4096, 26, 100_000, 16
    rows = (np.arange(F)[None, :] * V + zipf(rng, (B, F), V, 1.2)).astype(np.int32)
    t = SparseTable(F * V, D, SparseAdam(1e-3), device=dev)
    t.mode = "scan"
    dout = torch.randn(B, F * D, device=dev)
    r = torch.from_numpy(rows.reshape(-1)).to(dev)
    return t, lambda: t.accumulate(r, None, B, F, dout, F * D, D, 0), rows


def case_c5(rng, dev):
    """config 5: the 91 staytime fields, B = 2048, hashed Zipf(1.2) ids over one 10 M x 32 table"""
    B, F, V, D = 2048, 91, 10_000_000, 32
    ids = zipf(rng, (B, F), 1 << 40, 1.2).astype(np.uint64)
    rows = ((ids * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(20)) % np.uint64(V)
    rows = rows.astype(np.int32)
    t = SparseTable(V, D, SparseAdam(1e-3), device=dev, max_touched=B * 400)
    dout = torch.randn(B, F * D, device=dev)
    r = torch.from_numpy(rows.reshape(-1)).to(dev)
    return t, lambda: t.accumulate(r, None, B, F, dout, F * D, D, 1), rows


def case_c4_hist_scan(rng, dev):
    """the config-4 history push as the single-GPU Trainer runs it (scan mode, prefer_scan)"""
    t, fn, ids = case_c4_hist(rng, dev)
    t.mode = "scan"
    return t, fn, ids


def case_c3_scan(rng, dev):
    """config 3's push in scan mode (no claims: the claim cost by difference)"""
    t, fn, rows = case_c3(rng, dev)
    t.mode = "scan"
    return t, fn, rows


CASES = {"c3_scan": case_c3_scan, "c5": case_c5, "c3": case_c3, "c4_hist": case_c4_hist, "c4_q": case_c4_q, "c2": case_c2,
         "c4_hist_scan": case_c4_hist_scan}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--only", default=",".join(CASES))
    args = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda")
    out = {}
    for name in args.only.split(","):
        rng = np.random.default_rng(0)
        t, fn, rows = CASES[name](rng, dev)
        fn(); t.step(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(args.reps):
            e0.record(); fn(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
            t.step(); torch.cuda.synchronize()
        out[name] = {"us_median": round(float(np.median(ts)), 2), "us_min": round(min(ts), 2),
                     "ids": int(rows.size), "unique_rows": int(len(np.unique(rows)))}
        del t
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
