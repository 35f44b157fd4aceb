"""InteractingLayer forward / backward time per shape (HIP events, one launch each, B samples),
for A/B runs of the kernel families: the compiled-in instantiations vs the generic kernels
(RS_IL_FORCE_GENERIC=1) -- e.g. whether the generic backward can replace bwd2_kernel for the
shapes whose bwd3 LDS does not fit.
    python tools/il_shape_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402

SHAPES = [(26, 16, 16, 2, 3), (26, 16, 16, 4, 2), (26, 16, 32, 2, 1), (26, 32, 32, 2, 2),
          (40, 16, 16, 2, 2), (40, 8, 8, 2, 1), (19, 8, 8, 2, 1), (26, 16, 128, 1, 1),
          (26, 16, 24, 3, 1)]


def main(B=2048):
    lib = _lib.load()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    s = stream_handle()
    for F, E, U, H, L in SHAPES:
        x = torch.rand(B, F, E, device=dev, generator=g) - 0.5
        W = (torch.rand(E, 4 * U, device=dev, generator=g) - 0.5) * 0.5
        b = torch.zeros(4 * U, device=dev)
        gm, bt = torch.ones(U, device=dev), torch.zeros(U, device=dev)
        y = torch.empty(B, F * U, device=dev)
        xs = torch.empty(max(L - 1, 1), B, F, U, device=dev)
        dy = torch.randn(B, F * U, device=dev, generator=g)
        dx = torch.empty_like(x)
        wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U))
        ws = torch.empty(wsn, device=dev)
        dp = torch.empty(int(lib.rs_il_param_count(E, U)), device=dev)
        wa = (ptr(W), ptr(b), ptr(gm), ptr(bt), 1e-14, 1, 0.0, 0)
        fwd = lambda: call("rs_il_fwd", s, ptr(x), B, F, E, U, H, L, *wa, ptr(y), F * U,  # noqa: E731
                           ptr(xs) if L > 1 else None)
        bwd = lambda: call("rs_il_bwd", s, ptr(x), ptr(xs) if L > 1 else None, ptr(dy), F * U, B,  # noqa: E731
                           F, E, U, H, L, *wa, ptr(dx), 0, ptr(dp), 0, ptr(ws), wsn)
        res = []
        for fn in (fwd, bwd):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / 20 * 1e3)
        print(f"F={F} E={E} U={U} H={H} L={L} B={B}: fwd {res[0]:.1f} us, bwd {res[1]:.1f} us",
              flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
