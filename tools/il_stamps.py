"""Diagnostic: per-phase cycle shares of the IL backward (build with -DRS_IL_STAMPS)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle
B, F, E, U, H, L = 4096, 26, 16, 16, 2, 3
lib = _lib.load()
st = torch.zeros(10, dtype=torch.int64, device="cuda")
lib.rs_il_debug_set_stamps.argtypes = [ctypes.c_void_p]
lib.rs_il_debug_set_stamps(ptr(st))
dev = torch.device("cuda")
x = torch.rand(B, F, E, device=dev) - 0.5
W = (torch.rand(E, 4 * U, device=dev) - 0.5) * 0.5
bias = torch.zeros(4 * U, device=dev); g = torch.ones(U, device=dev); be = torch.zeros(U, device=dev)
xs = torch.empty(L - 1, B, F, U, device=dev); y = torch.empty(B, F * U, device=dev)
dy = torch.randn(B, F * U, device=dev); dx = torch.empty_like(x)
wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U)); ws = torch.empty(wsn, device=dev)
s = stream_handle()
SAVED = os.environ.get("IL_STAMPS_SAVED", "1") == "1"   # bwd4 (saved pair) or bwd3
ns = int(lib.rs_il_attn_save_floats(B, F, U, H, L))
asave = torch.empty(max(ns, 1), device=dev)
call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, L, ptr(W), ptr(bias), ptr(g), ptr(be), 1e-14, 1, 0.0, 0, ptr(y), F * U, ptr(xs), ptr(asave), ns)
for _ in range(3):
    if SAVED:
        call("rs_il_bwd_saved", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(g), ptr(be), 1e-14, 1, 0.0, 0, ptr(dx), 0, None, 0, ptr(ws), wsn, ptr(asave), ns)
    else:
        call("rs_il_bwd", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(g), ptr(be), 1e-14, 1, 0.0, 0, ptr(dx), 0, None, 0, ptr(ws), wsn)
torch.cuda.synchronize()
v = st.cpu().tolist()[:10]
names = (["wait x/save (it<L-1)", "P1 proj + xa", "P3 LN bwd", "Q-pass", "K-pass", "G-Q", "dW (MFMA)",
          "dx it>0", "dx+push it=0", "wait (sample start)"] if SAVED else
         ["x load/prefetch", "projection(MFMA)", "attn recompute", "LN bwd", "dV", "dS/dQ", "dK + G", "dW (MFMA)", "dx (MFMA) it>0", "dx+push it=0"])
tot = sum(v)
for n, c in zip(names, v):
    print(f"{n:18s} {100.0 * c / tot:6.1f}%")
