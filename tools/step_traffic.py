"""Per-kernel HBM traffic of the config-2 step from rocprofv3 PMC passes over a short bench run
(tools/r04_final_b.sh): FETCH_SIZE and WRITE_SIZE in separate passes, per mode (the deferred dW1
default "dz" and the round-3 form "part" = RS_HEAD_W1_PARTIALS=1).  FETCH_SIZE x2 (gfx950 reports
half of wide coalesced reads, MI355X_MICROARCH.md), WRITE_SIZE as is; KB per dispatch.
    python tools/step_traffic.py gpurun_out/r04_final out.json"""
import collections
import csv
import glob
import json
import sys

KERNELS = ("wfwd_kernel", "head_train_kernel", "bwd4_kernel", "wbwd_kernel",
           "partials_reduce_adam_kernel")


def per_kernel(root, mode, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{root}/step_{mode}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for k in KERNELS:
                if k in r["Kernel_Name"]:
                    vals[k].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main(root, out):
    res = {"correction": "FETCH_SIZE x2 + WRITE_SIZE, KB per dispatch -> MB",
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                     "bench.py --steps 5 --warmup 2 (config 2, B = 4096); dispatches include the "
                     "warm-up / capture replays"}
    for mode in ("dz", "part"):
        fe, wr = per_kernel(root, mode, "FETCH_SIZE"), per_kernel(root, mode, "WRITE_SIZE")
        m = {}
        for k in KERNELS:
            if k in fe and k in wr:
                m[k] = {"fetch_mb": round(2 * fe[k][0] / 1024, 2), "write_mb": round(wr[k][0] / 1024, 2),
                        "hbm_mb": round((2 * fe[k][0] + wr[k][0]) / 1024, 2),
                        "dispatches": [fe[k][1], wr[k][1]]}
        m["step_total_mb"] = round(sum(v["hbm_mb"] for v in m.values()), 2)
        res[mode] = m
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
