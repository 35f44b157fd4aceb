"""rs_dense_fwd / rs_dense_bwd_weight (the HIP GEMM engine) vs torch.mm (rocBLAS / hipBLASLt)
on the config-3/5 GEMM shapes, fp32, HIP events."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402


def t_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    s = stream_handle()
    for M, K, N in ((2048, 1712, 960), (2048, 1840, 400), (4096, 1616, 273), (2048, 224, 1152),
                    (2048, 528, 400), (2048, 1712, 256), (4096, 1600, 32)):
        X = torch.randn(M, K, device=dev)
        W = torch.randn(K, N, device=dev) * 0.02
        b = torch.zeros(N, device=dev)
        Y = torch.empty(M, N, device=dev)
        dY = torch.randn(M, N, device=dev)
        dW = torch.empty(K, N, device=dev)
        db = torch.empty(N, device=dev)
        wsn = int(lib.rs_dense_bwd_weight_workspace_floats(M, K, N))
        ws = torch.empty(max(wsn, 1), device=dev)
        ours_f = t_us(lambda: call("rs_dense_fwd", s, ptr(X), M, K, K, ptr(W), ptr(b), N, 0, ptr(Y), N))
        blas_f = t_us(lambda: torch.mm(X, W, out=Y))
        ours_w = t_us(lambda: call("rs_dense_bwd_weight", s, ptr(X), K, ptr(dY), N, ptr(dY), N, 0, M,
                                   K, N, ptr(dW), ptr(db), 0, ptr(ws), wsn))
        blas_w = t_us(lambda: torch.mm(X.t(), dY, out=dW))
        dX = torch.empty(M, K, device=dev)
        ours_d = t_us(lambda: call("rs_dense_bwd_data", s, ptr(dY), N, ptr(dY), N, 0, ptr(W), M, K, N,
                                   ptr(dX), K, 0))
        blas_d = t_us(lambda: torch.mm(dY, W.t(), out=dX))
        fl = 2 * M * K * N
        print(json.dumps({"M": M, "K": K, "N": N, "fwd_us": round(ours_f, 1), "blas_fwd_us": round(blas_f, 1),
                          "wgrad_us": round(ours_w, 1), "blas_wgrad_us": round(blas_w, 1),
                          "dgrad_us": round(ours_d, 1), "blas_dgrad_us": round(blas_d, 1),
                          "fwd_tf": round(fl / ours_f / 1e6, 1), "blas_fwd_tf": round(fl / blas_f / 1e6, 1)}))


if __name__ == "__main__":
    main()
