"""HBM traffic of the InteractingLayer backward + fused push (the launch bench.py times) from the
rocprofv3 PMC passes of tools/profile_round.sh (FETCH_SIZE and WRITE_SIZE in separate passes over
IL_BENCH_ONLY=push_hot_base_saved tools/il_bench.py: one bwd4 launch kind per pass).
MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950
(x2 correction); WRITE_SIZE is exact for 16-B streaming stores.  Both are in KB per dispatch.
    python tools/traffic_json.py gpurun_out/r01 profiles/il_bwd_traffic.json"""
import csv
import glob
import json
import sys

B, F, E, U, L = 4096, 26, 16, 16, 3
GRID, NPARAM = 512, 1120  # kBwd3Grid blocks, per-block parameter partial row
# algorithmic bytes of one rs_il_bwd_push launch (dparams NULL): read x (B F E), xsave
# ((L-1) B F U), dy (B F U), the head's share dx_base (B F E), the rows (B F int32); add dL/dx0
# into the table (B F E floats) and mark the flags (B F int32); write the per-block partials
# v4 (saved path) also reads the forward's attention save: O [F U] + softmax stats [2 H F] per
# (iteration, sample), padded to 4 floats (il_kernels.hpp small_save_stride)
H = 2
SV = (F * U + 2 * H * F + 3) & ~3
ALG = 4 * (B * F * E + (L - 1) * B * F * U + B * F * U + B * F * E + B * F + B * F * E + B * F) \
    + 4 * GRID * NPARAM + 4 * L * B * SV


def mean_counter(root, name, kernel_sub):
    vals = []
    for f in glob.glob(f"{root}/pmc_{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and kernel_sub in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main(root, out):
    k = "bwd4_kernel"
    fetch, n1 = mean_counter(root, "FETCH_SIZE", k)
    write, n2 = mean_counter(root, "WRITE_SIZE", k)
    res = {
        "kernel": "rs_il::bwd4_kernel<Cfg<16,16,2,26,true,false>,false> via rs_il_bwd_push_saved "
                  "(B=4096, F=26, E=U=16, H=2, L=3; hot rows, head share added)",
        "hbm_bytes_per_launch": round((2 * fetch + write) * 1024) if fetch and write else None,
        "fetch_size_kb": fetch, "write_size_kb": write, "dispatches": [n1, n2],
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads; "
                      "MI355X_MICROARCH.md HBM), WRITE_SIZE as is; both KB per dispatch",
        "algorithmic_bytes_per_launch": ALG,
        "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) "
                  "over IL_BENCH_ONLY=push_hot_base_saved tools/il_bench.py",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
