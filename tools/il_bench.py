"""Time the InteractingLayer kernels alone at config-2 size (B=4096, F=26, E=U=16, H=2, L=3)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommendsystem_amd import _lib
from recommendsystem_amd._lib import call, ptr, stream_handle

def main(B=4096, F=26, E=16, U=16, H=2, L=3, reps=50):
    lib = _lib.load()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.rand(B, F, E, device=dev, generator=g) - 0.5)
    W = (torch.rand(E, 4 * U, device=dev, generator=g) - 0.5) * 0.5
    bias = torch.zeros(4 * U, device=dev); gamma = torch.ones(U, device=dev); beta = torch.zeros(U, device=dev)
    y = torch.empty(B, F * U, device=dev); xs = torch.empty(max(L - 1, 1), B, F, U, device=dev)
    dy = torch.randn(B, F * U, device=dev, generator=g); dx = torch.empty_like(x)
    wsn = int(lib.rs_il_bwd_workspace_floats(B, E, U)); ws = torch.empty(wsn, device=dev)
    dp = torch.empty(int(lib.rs_il_param_count(E, U)), device=dev)
    s = stream_handle()
    fwd = lambda: call("rs_il_fwd", s, ptr(x), B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(y), F * U, ptr(xs))
    bwd = lambda: call("rs_il_bwd", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(dx), 0, None, 0, ptr(ws), wsn)
    red = lambda: call("rs_il_bwd", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(dx), 0, ptr(dp), 0, ptr(ws), wsn)
    # fused push variants (the trainer's launch): uniform rows (no hot rows) and Zipf-like rows
    # (1/3 of the ids on one row per field), with and without the head's dx share to add
    T = 26 * 100_000
    rows_u = (torch.arange(B * F, device=dev, dtype=torch.int32) * 7919) % T
    hot = torch.rand(B * F, device=dev, generator=g) < 0.33
    rows_z = torch.where(hot, (torch.arange(B * F, device=dev) % F).to(torch.int32) * 100_000, rows_u)
    table = torch.zeros(T, E, device=dev); flag = torch.full((T,), -1, dtype=torch.int32, device=dev)
    base = torch.randn(B, F * E, device=dev, generator=g)
    def push(rows, bp):
        return lambda: call("rs_il_bwd_push", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(bp), ptr(rows), ptr(table), ptr(flag), None, 0, ptr(ws), wsn)
    ns = int(lib.rs_il_attn_save_floats(B, F, U, H, L))
    asave = torch.empty(max(ns, 1), device=dev)
    fwd_s = lambda: call("rs_il_fwd_saved", s, ptr(x), B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(y), F * U, ptr(xs), ptr(asave), ns)
    bwd_s = lambda: call("rs_il_bwd_saved", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(dx), 0, None, 0, ptr(ws), wsn, ptr(asave), ns)
    def push_s(rows, bp):
        return lambda: call("rs_il_bwd_push_saved", s, ptr(x), ptr(xs), ptr(dy), F * U, B, F, E, U, H, L, ptr(W), ptr(bias), ptr(gamma), ptr(beta), 1e-14, 1, 0.0, 0, ptr(bp), ptr(rows), ptr(table), ptr(flag), None, 0, ptr(ws), wsn, ptr(asave), ns)
    fwd_s(); torch.cuda.synchronize()
    out = {}
    only = os.environ.get("IL_BENCH_ONLY")  # one variant (PMC passes: one kernel per dispatch kind)
    for name, fn in (("fwd", fwd), ("bwd", bwd), ("bwd+reduce", red), ("push_uniform", push(rows_u, None)),
                     ("push_uniform_base", push(rows_u, base)), ("push_hot_base", push(rows_z, base)),
                     ("fwd_saved", fwd_s), ("bwd_saved", bwd_s), ("push_hot_base_saved", push_s(rows_z, base))):
        if only and name != only:
            continue
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): fn()
        e1.record(); torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    fl = 289_536 * B
    if "fwd_us" in out:
        out["fwd_tflops"] = round(fl / out["fwd_us"] / 1e6, 2)
    if "bwd_us" in out:
        out["bwd_tflops"] = round(2 * fl / out["bwd_us"] / 1e6, 2)
    print(json.dumps(out))

if __name__ == "__main__":
    main(reps=int(os.environ.get("REPS", "50")))
