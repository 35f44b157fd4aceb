"""Diagnostic: per-phase cycles of the InteractingLayer kernels (build with -DRS_IL_STAMPS:
RS_LIB_OUT=recommendsystem_amd/librecsys_amd_stamps.so python -m recommendsystem_amd.build
-DRS_IL_STAMPS, run with RS_LIB_PATH pointing at it).  Prints, per batch size and variant, the
average s_memtime cycles per wave per sample-iteration spent in each phase (stamps summed over
every wave of the launch), i.e. the latency budget of one sample's chain."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle

F, E, U, H, L = 26, 16, 16, 2, 3
lib = _lib.load()
st = torch.zeros(10, dtype=torch.int64, device="cuda")
lib.rs_il_debug_set_stamps.argtypes = [ctypes.c_void_p]
lib.rs_il_debug_set_stamps(ptr(st))
dev = torch.device("cuda")
REPS = 5
FWD = ["load x / gather", "projection", "attention", "LN epilogue"]
BWD = ["wait x/save", "P1 proj + xa", "P3 LN bwd", "Q-pass", "K-pass", "P7 dW/dx", "dx sum it>0",
       "dx push it=0"]
for B in [int(b) for b in os.environ.get("BATCHES", "512 4096").split()]:
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(B, F, E, device=dev, generator=g) - 0.5
    W = (torch.rand(E, 4 * U, device=dev, generator=g) - 0.5) * 0.5
    bias = torch.zeros(4 * U, device=dev); gm = torch.ones(U, device=dev); be = torch.zeros(U, device=dev)
    xs = torch.empty(L - 1, B, F, U, device=dev); y = torch.empty(B, F * U, device=dev)
    dy = torch.randn(B, F * U, device=dev, generator=g); dx = torch.empty_like(x)
    wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U)); ws = torch.empty(wsn, device=dev)
    ns = int(lib.rs_il_attn_save_floats(B, F, U, H, L)); asave = torch.empty(ns, device=dev)
    s = stream_handle()
    for variant in os.environ.get("VARIANTS", "wide wave").split():
        with _lib.il_variant(variant):
            fwd = lambda: call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, L, ptr(W), ptr(bias),
                               ptr(gm), ptr(be), 1e-14, 1, 0.0, 0, ptr(y), F * U, ptr(xs), ptr(asave), ns)
            bwd = lambda: call("rs_il_bwd_saved", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L,
                               ptr(W), ptr(bias), ptr(gm), ptr(be), 1e-14, 1, 0.0, 0, ptr(dx), 0, None,
                               0, ptr(ws), wsn, ptr(asave), ns)
            for name, fn, names in (("fwd", fwd, FWD), ("bwd", bwd, BWD)):
                fn(); torch.cuda.synchronize()
                st.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(REPS):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / REPS
                v = st.cpu().tolist()
                # waves per launch: wide = 4 per sample; wave variant = one wave per sample
                waves = (4 if variant == "wide" else 1) * B
                per = REPS * waves * L
                tot = sum(v)
                # per-wave wall cycles of the whole launch vs the launch time: the implied clock
                per_wave_launch = tot / (REPS * waves)
                print(f"B={B} {variant} {name}: {tot / per:8.0f} cycles per wave per sample-iteration; "
                      f"launch {us:.1f} us, per-wave stamped span {per_wave_launch:.0f} cycles "
                      f"(= {per_wave_launch / us / 1e3:.2f} GHz if the span were the launch)")
                for n, c in zip(names, v):
                    print(f"    {n:16s} {c / per:8.0f}  {100.0 * c / max(tot, 1):5.1f}%")
