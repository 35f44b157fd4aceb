"""Time the fused AutoInt head kernel (rs_mlp_head_train) alone at config 2 ([416 -> 32 -> 16] +
[432 -> 1], B = 4096 and 512), optionally from a variant library (RS_LIB_PATH, built with
RS_LIB_OUT and -DRS_HEAD_SKIP=bits: a phase-share breakdown, not a correct head)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from recommendsystem_amd import _lib  # noqa: E402
from recommendsystem_amd._lib import call, ptr, stream_handle  # noqa: E402


def bench(B, K0=416, S=416, N1=32, N2=16, reps=200):
    lib = _lib.load()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev, generator=g) - 0.5) * 0.2  # noqa: E731
    x0, il = r(B, K0), r(B, S)
    W1, b1, W2, b2 = r(K0, N1), r(N1), r(N1, N2), r(N2)
    W3, b3 = r(N2 + S, 1), r(1)
    y = (torch.rand(B, 1, device=dev, generator=g) < 0.25).float()
    p = torch.empty(B, 1, device=dev)
    dil, dx0 = torch.empty(B, S, device=dev), torch.empty(B, K0, device=dev)
    wsn = int(lib.rs_mlp_head_workspace_floats(B, K0, N1, N2, S, 1))
    ws = torch.empty(wsn, device=dev)
    s = stream_handle()
    fn = lambda: call("rs_mlp_head_train", s, ptr(x0), K0, ptr(il), S, B, K0, S, N1, 1, N2, 1, 1, 2,  # noqa: E731
                      ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(W3), ptr(b3), ptr(y), 1e-6, 1.0, 1e-6,
                      ptr(p), ptr(dil), S, ptr(dx0), K0, 0, ptr(ws), wsn)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    if os.environ.get("HEAD_STAMPS"):  # -DRS_HEAD_STAMPS build: block 0's phase cycles in d il row 0
        fn()
        torch.cuda.synchronize()
        return us, [int(v) for v in dil[0, :8].tolist()]
    return us


if __name__ == "__main__":
    print(json.dumps({"lib": os.environ.get("RS_LIB_PATH", "default"),
                      "b4096_us": bench(4096), "b512_us": bench(512)}))
