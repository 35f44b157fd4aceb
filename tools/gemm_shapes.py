"""Every rs_dense_* GEMM one eager train step of a configs-3/5 workload launches (shape, operand
mode, calls per step), then each distinct shape timed alone with HIP events against torch.mm
(hipBLASLt / rocBLAS) on the same fp32 operands.  Prints one JSON line per shape and a total.

    python tools/gemm_shapes.py --workload staytime [--batch 2048]"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402

SEEN = collections.Counter()


class _Rec:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if name == "rs_dense_fwd":
            def w(*a):
                SEEN[("fwd", a[2], a[3], a[7], a[8])] += 1   # M, K, N, act
                return fn(*a)
            return w
        if name == "rs_dense_bwd_data":
            def w(*a):
                SEEN[("bwd_data", a[7], a[8], a[9], a[5])] += 1  # M, K, N, act
                return fn(*a)
            return w
        if name == "rs_dense_bwd":
            def w(*a):
                SEEN[("bwd", a[9], a[10], a[11], a[7])] += 1  # M, K, N, act
                return fn(*a)
            return w
        if name == "rs_dense_bwd_weight":
            def w(*a):
                SEEN[("bwd_weight", a[8], a[9], a[10], a[7])] += 1  # M, K, N, act
                return fn(*a)
            return w
        return fn


def t_us(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def one_step(workload, B):
    from recommendsystem_amd import workloads as W
    from recommendsystem_amd.models import MultiHeadConfig, MultiHeadRanker
    from recommendsystem_amd.trainer import Trainer
    dev = torch.device("cuda")
    rng = np.random.default_rng(10)
    if workload == "multi_head":
        cfg = MultiHeadConfig()
        model = MultiHeadRanker(cfg, device=dev, seed=0)
        tr = Trainer(model, cfg.lr_dense, model.tables())
        batch = W.multi_head_batch(rng, B, cfg, dev)
    else:
        model = W.StaytimeRoughRank(device=dev, seed=0)
        tr = Trainer(model, 5e-4, [model.table], lr_groups=[(model.dssm, model.rr_cfg.lr_dense)])
        batch = W.staytime_batch(rng, B, model, dev)
    tr.step(*batch)
    torch.cuda.synchronize()
    SEEN.clear()
    tr.step(*batch)
    torch.cuda.synchronize()


def time_shape(kind, M, K, N, act):
    dev = torch.device("cuda")
    s = stream_handle()
    lib = _lib.load()
    X = torch.randn(M, K, device=dev)
    Wt = torch.randn(K, N, device=dev) * 0.05
    b = torch.zeros(N, device=dev)
    Y = torch.rand(M, N, device=dev)
    dY = torch.randn(M, N, device=dev)
    if kind == "fwd":
        ours = t_us(lambda: call("rs_dense_fwd", s, ptr(X), M, K, K, ptr(Wt), ptr(b), N, act, ptr(Y), N))
        blas = t_us(lambda: torch.mm(X, Wt, out=Y))
    elif kind == "bwd_data":
        dX = torch.empty(M, K, device=dev)
        ours = t_us(lambda: call("rs_dense_bwd_data", s, ptr(dY), N, ptr(Y), N, act, ptr(Wt), M, K, N,
                                 ptr(dX), K, 0))
        blas = t_us(lambda: torch.mm(dY, Wt.t(), out=dX))
    elif kind == "bwd":
        dX = torch.empty(M, K, device=dev)
        dW = torch.empty(K, N, device=dev)
        db = torch.empty(N, device=dev)
        wsn = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
        ws = torch.empty(max(wsn, 1), device=dev)
        ours = t_us(lambda: call("rs_dense_bwd", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, ptr(Wt), M,
                                 K, N, ptr(dX), K, 0, ptr(dW), ptr(db), 0, ptr(ws), wsn))
        blas = t_us(lambda: (torch.mm(dY, Wt.t(), out=dX), torch.mm(X.t(), dY, out=dW)))
    else:
        dW = torch.empty(K, N, device=dev)
        db = torch.empty(N, device=dev)
        wsn = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
        ws = torch.empty(max(wsn, 1), device=dev)
        ours = t_us(lambda: call("rs_dense_bwd_weight", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, M,
                                 K, N, ptr(dW), ptr(db), 0, ptr(ws), wsn))
        blas = t_us(lambda: torch.mm(X.t(), dY, out=dW))
    return ours, blas


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="staytime")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--min-macs", type=float, default=0, help="time only shapes this large")
    a = ap.parse_args()
    B = a.batch or (2048 if a.workload == "staytime" else 4096)
    lib = _lib.load()
    _lib._LIB = _Rec(lib)
    one_step(a.workload, B)
    _lib._LIB = lib
    tot_o = tot_b = 0.0
    for (kind, M, K, N, act), n in sorted(SEEN.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3] * kv[1]):
        if M * K * N < a.min_macs:
            continue
        o, bl = time_shape(kind, M, K, N, act)
        tot_o += o * n
        tot_b += bl * n
        fl = 2.0 * M * K * N
        print(json.dumps({"kind": kind, "M": M, "K": K, "N": N, "act": act, "calls": n,
                          "us": round(o, 1), "blas_us": round(bl, 1), "tf": round(fl / o / 1e6, 1),
                          "blas_tf": round(fl / bl / 1e6, 1)}), flush=True)
    print(json.dumps({"workload": a.workload, "batch": B, "gemm_us_per_step": round(tot_o, 1),
                      "blas_us_per_step": round(tot_b, 1), "launches": sum(SEEN.values()),
                      "tune": os.environ.get("RS_GEMM_TUNE"), "tile": os.environ.get("RS_GEMM_BIG_TILE")}),
          flush=True)


if __name__ == "__main__":
    main()
