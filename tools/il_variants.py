"""Diagnostic: time the wide InteractingLayer kernels with phases dropped (tools/il_variants.hip,
il_wide.hpp SKIP bits), HIP events per launch, config-2 shape, B from $BATCHES.
Build (CPU container): python3 tools/il_variants.py build ; run on the GPU box: python3 tools/il_variants.py"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "_gpuvar", "libilvar.so")  # (tools/_bin does not travel to the box)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "--offload-arch=gfx950", "-munsafe-fp-atomics",
                           os.path.join(ROOT, "tools", "il_variants.hip"), "-o", LIB])
    sys.exit(0)
import torch
lib = ctypes.CDLL(LIB)
F, E, U, H, L = 26, 16, 16, 2, 3
dev = torch.device("cuda")
vp = ctypes.c_void_p
P = lambda t: ctypes.c_void_p(t.data_ptr())
FWD = {0: "full", 1: "-proj", 2: "-attn", 4: "-LN", 8: "-load", 3: "-proj-attn", 7: "load only"}
BWD = {0: "full", 1: "-P1", 2: "-P3", 4: "-Q", 8: "-K", 12: "-Q-K", 16: "-P7", 32: "-dxsum", 63: "skeleton"}
for B in [int(b) for b in os.environ.get("BATCHES", "512 4096").split()]:
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(B, F, E, device=dev, generator=g) - 0.5
    W = (torch.rand(E, 4 * U, device=dev, generator=g) - 0.5) * 0.5
    b = torch.zeros(4 * U, device=dev); gm = torch.ones(U, device=dev); be = torch.zeros(U, device=dev)
    xs = torch.empty(L - 1, B, F, U, device=dev); y = torch.empty(B, F * U, device=dev)
    asave = torch.zeros(L * B * (F * U + 2 * H * F + 4), device=dev)
    dy = torch.randn(B, F * U, device=dev, generator=g); dx = torch.empty_like(x)
    ws = torch.empty(1024 * 1120, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    def tm(fn, reps=50):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record(); torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps
    lib.ilvar_fwd(0, s, P(x), P(W), P(b), P(gm), P(be), P(y), P(xs), P(asave), ctypes.c_int64(B))
    for k, n in FWD.items():
        t = tm(lambda: lib.ilvar_fwd(k, s, P(x), P(W), P(b), P(gm), P(be), P(y), P(xs), P(asave), ctypes.c_int64(B)))
        print(f"B={B} fwd {n:12s} {t:8.2f} us")
    lib.ilvar_fwd(0, s, P(x), P(W), P(b), P(gm), P(be), P(y), P(xs), P(asave), ctypes.c_int64(B))
    torch.cuda.synchronize()
    for k, n in BWD.items():
        t = tm(lambda: lib.ilvar_bwd(k, s, P(x), P(xs), P(dy), P(W), P(b), P(gm), P(be), P(dx), P(ws), P(asave), ctypes.c_int64(B)))
        print(f"B={B} bwd {n:12s} {t:8.2f} us")
