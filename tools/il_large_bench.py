"""Time the many-field InteractingLayer kernels at config-3 size (B=4096, F=200, E=U=8, H=2, L=1,
dropout 0.2): forward and backward (rs_il_fwd / rs_il_bwd, HIP events)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402


def main(B=4096, F=200, E=8, U=8, H=2, reps=10, drop=0.2):
    lib = _lib.load()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, F, E, device=dev, generator=g) - 0.5
    W = (torch.rand(E, 4 * U, device=dev, generator=g) - 0.5) * 0.5
    b, gm, bt = torch.zeros(4 * U, device=dev), torch.ones(U, device=dev), torch.zeros(U, device=dev)
    y = torch.empty(B, F * U, device=dev)
    dy = torch.randn(B, F * U, device=dev, generator=g)
    dx = torch.empty_like(x)
    wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U))
    ws = torch.empty(wsn, device=dev)
    s = stream_handle()
    fwd = lambda: call("rs_il_fwd", s, ptr(x), B, F, E, U, H, 1, ptr(W), ptr(b), ptr(gm), ptr(bt), 1e-14, 1,  # noqa: E731
                       drop, 3, ptr(y), F * U, None)
    bwd = lambda: call("rs_il_bwd", s, ptr(x), None, ptr(dy), F * U, B, F, E, U, H, 1, ptr(W), ptr(b),  # noqa: E731
                       ptr(gm), ptr(bt), 1e-14, 1, drop, 3, ptr(dx), 0, None, 0, ptr(ws), wsn)
    ns = int(lib.rs_il_attn_save_floats(B, F, U, H, 1))
    asave = torch.empty(ns, device=dev)
    fwds = lambda: call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, 1, ptr(W), ptr(b), ptr(gm),  # noqa: E731
                        ptr(bt), 1e-14, 1, drop, 3, ptr(y), F * U, None, ptr(asave), ns)
    bwds = lambda: call("rs_il_bwd_saved", s, ptr(x), None, ptr(dy), F * U, B, F, E, U, H, 1,  # noqa: E731
                        ptr(W), ptr(b), ptr(gm), ptr(bt), 1e-14, 1, drop, 3, ptr(dx), 0, None, 0,
                        ptr(ws), wsn, ptr(asave), ns)
    out = {}
    for name, fn in (("fwd", fwd), ("bwd", bwd), ("fwd_saved", fwds), ("bwd_saved", bwds)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 1)
    fl = 1_382_400 * B
    out["fwd_tflops"] = round(fl / out["fwd_us"] / 1e6, 2)
    out["bwd_tflops"] = round(2 * fl / out["bwd_us"] / 1e6, 2)
    out["bwd_saved_tflops"] = round(2 * fl / out["bwd_saved_us"] / 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
