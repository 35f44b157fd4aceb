"""Host-side probe of the C ABI, run by tests/test_asan_host.py in a subprocess with the
AddressSanitizer runtime preloaded, against librecsys_amd built with -Xarch_host
-fsanitize=address (host code instrumented, device code unchanged).  No GPU is needed: it calls

  * every size / plan query (workspace sizes, partial-row counts, dry-run dispatches such as
    rs_il_bwd_partial_blocks / rs_il_bwd_xt_supported, the GEMM planner behind the grouped
    workspace query) over a grid of shapes, including zero, negative and extreme values;
  * every stream entry point with null pointers and zero / negative / positive sizes (argument
    validation must reject them or return without launching);
  * the grouped Dense entry points with host descriptor arrays of 0 .. 9 layers.

Any out-of-bounds host access, use-after-free or crash ends the process with a sanitizer report
(nonzero exit).  Usage: python tests/asan_host_probe.py LIB include/recsys_amd.h
"""
import ctypes
import itertools
import re
import sys

C_TYPES = {"int": ctypes.c_int, "int64_t": ctypes.c_int64, "uint64_t": ctypes.c_uint64,
           "int32_t": ctypes.c_int32, "uint32_t": ctypes.c_uint32,
           "float": ctypes.c_float, "double": ctypes.c_double}


def prototypes(header):
    src = re.sub(r"/\*.*?\*/", "", open(header).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(int|int64_t)\s+(rs_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = []
        for a in m.group(3).split(","):
            a = " ".join(a.split())
            if a in ("", "void"):
                continue
            if "*" in a:
                args.append("ptr")
            else:
                args.append(a.rsplit(" ", 1)[0].replace("const ", ""))
        out[m.group(2)] = (m.group(1), args)
    return out


def main(lib_path, header):
    lib = ctypes.CDLL(lib_path)
    protos = prototypes(header)
    n_calls = 0
    for name, (ret, args) in sorted(protos.items()):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int64 if ret == "int64_t" else ctypes.c_int
        fn.argtypes = [ctypes.c_void_p if a == "ptr" else C_TYPES[a] for a in args]
    # ---- size / plan queries over a grid of shapes ----
    dims = [0, 1, 3, 8, 16, 26, 32, 64, 65, 128, 200, 256, 257]
    for B in (0, 1, 7, 512, 1536, 1537, 4096, 100_000, -1):
        for F, E, U, H in itertools.product((1, 4, 26, 37, 64, 65, 200, 256, 300),
                                            (8, 16, 32), (8, 16, 24, 64, 128), (1, 2, 3, 4)):
            ws = lib.rs_il_bwd_workspace_floats(B, E, U)
            for w in (ws, 0, -5):
                lib.rs_il_bwd_partial_blocks(B, F, E, U, H, w)
                lib.rs_il_bwd_saved_partial_blocks(B, F, E, U, H, w)
                lib.rs_il_bwd_xt_supported(B, F, E, U, H, w)
                n_calls += 3
            lib.rs_il_attn_save_floats(B, F, U, H, 3)
            lib.rs_il_param_count(E, U)
        lib.rs_il_xt_splits(B)
        lib.rs_mlp_head_partial_blocks(B)
        for K0, N1, N2, S, T in ((416, 32, 16, 416, 1), (416, 64, 0, 416, 4), (16, 16, 16, 16, 2),
                                 (0, 0, 0, 0, 0), (-1, 32, 16, 416, 1)):
            lib.rs_mlp_head_param_floats(K0, N1, N2, S, T)
            lib.rs_mlp_head_workspace_floats(B, K0, N1, N2, S, T)
            lib.rs_mlp_head_dz_workspace_floats(B, K0, N1, N2, S, T)
        for K, N in itertools.product(dims, dims):
            lib.rs_dense_bwd_weight_workspace_floats(B, K, N)
            n_calls += 1
        for F in (0, 1, 26, 91, 1000):
            lib.rs_sparse_push_workspace_bytes(B, F)
            lib.rs_sparse_sorted_workspace_bytes(B * max(F, 1))
        for world in (0, 1, 2, 8, 1024, 1025):
            lib.rs_owner_route_workspace_bytes(B, world)
        for T, Hh in ((0, 0), (100, 16), (50, 32), (1, 1)):
            for variant in (0, 1, 2):
                lib.rs_din_param_count(variant, Hh)
                lib.rs_din_bwd_workspace_floats(variant, B, T, Hh)
        lib.rs_cross_bwd_workspace_floats(B, 64, 3)
        lib.rs_ffm_param_count(4, 4, 16, 8)
        lib.rs_ffm_bwd_workspace_floats(B, 4, 4, 16, 8)
        lib.rs_grouped_head_bwd_workspace_floats(B, 7, 32)
        lib.rs_field_linear_workspace_floats(B, 16, 175, 8)
        lib.rs_fm_proj_workspace_floats(B, 64, 8)
    for nthr in (-1, 0, 2, 3, 200, 1024, 1025):
        lib.rs_ctr_metrics_state_doubles(nthr)
    # ---- grouped Dense: host descriptor arrays (the GEMM planner reads them) ----
    for G in range(0, 10):
        for M, K, N in ((0, 0, 0), (2048, 1712, 256), (5, 3, 7), (4096, 16, 1)):
            fwd = (ctypes.c_int64 * max(10 * G, 1))(*([M, K, N, K, N, 1, 0, 0, 0, 0] * G))
            bwdd = (ctypes.c_int64 * max(12 * G, 1))(*([M, K, N, N, N, 1, 0, 0, 0, 0, K, 0] * G))
            bwdw = (ctypes.c_int64 * max(13 * G, 1))(*([M, K, N, K, N, N, 1, 0, 0, 0, 0, 0, 0] * G))
            lib.rs_dense_fwd_grouped(None, G, fwd)
            lib.rs_dense_bwd_data_grouped(None, G, bwdd)
            wsn = lib.rs_dense_bwd_weight_grouped_workspace_floats(G, bwdw)
            lib.rs_dense_bwd_weight_grouped(None, G, bwdw, None, max(wsn, 0))
            n_calls += 4
    # ---- every stream entry point with null pointers and degenerate sizes ----
    skip = {"rs_dense_fwd_grouped", "rs_dense_bwd_data_grouped", "rs_dense_bwd_weight_grouped",
            "rs_dense_bwd_weight_grouped_workspace_floats"}
    for name, (ret, args) in sorted(protos.items()):
        if name in skip or not args or args[0] != "ptr":
            continue
        fn = getattr(lib, name)
        for fill in (0, -1, 1, 7):
            vals = [None if a == "ptr" else (float(fill) if a in ("float", "double") else
                                             (fill if a != "uint64_t" else abs(fill)))
                    for a in args]
            fn(*vals)
            n_calls += 1
    print(f"asan host probe: {len(protos)} entry points, {n_calls}+ calls, no sanitizer report")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
