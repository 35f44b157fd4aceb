"""Run one large Dense product REPS times (profiling target): python tools/gemm_one.py FORM M K N [act]
FORM: fwd | data | weight (rs_dense_fwd / rs_dense_bwd_data / rs_dense_bwd_weight)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402


def main(form, M, K, N, act=0, reps=20):
    lib = _lib.load()
    dev = torch.device("cuda")
    s = stream_handle()
    X = torch.randn(M, K, device=dev)
    W = torch.randn(K, N, device=dev) * 0.02
    b = torch.zeros(N, device=dev)
    Y = torch.rand(M, N, device=dev)
    dY = torch.randn(M, N, device=dev)
    dX = torch.empty(M, K, device=dev)
    dW = torch.empty(K, N, device=dev)
    db = torch.empty(N, device=dev)
    wsn = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
    ws = torch.empty(max(wsn, 1), device=dev)
    if form == "fwd":
        fn = lambda: call("rs_dense_fwd", s, ptr(X), M, K, K, ptr(W), ptr(b), N, act, ptr(Y), N)
    elif form == "data":
        fn = lambda: call("rs_dense_bwd_data", s, ptr(dY), N, ptr(Y), N, act, ptr(W), M, K, N, ptr(dX), K, 0)
    else:
        fn = lambda: call("rs_dense_bwd_weight", s, ptr(X), K, ptr(dY), N, ptr(Y), N, act, M, K, N,
                          ptr(dW), ptr(db), 0, ptr(ws), wsn)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{form} {M}x{K}x{N} act {act}: {a.elapsed_time(e) / reps * 1e3:.1f} us")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]), int(a[2]), int(a[3]), int(a[4]) if len(a) > 4 else 0)
