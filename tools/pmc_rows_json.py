"""Per-(kernel, grid) HBM traffic from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_rows.sh:
bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE, KB -> bytes (MI355X_MICROARCH.md HBM section:
gfx950 FETCH_SIZE reports half of wide coalesced reads, WRITE_SIZE exact for 16-B stores).
    python tools/pmc_rows_json.py gpurun_out/pmc_rows  ->  <dir>/traffic.json"""
import collections
import csv
import glob
import json
import sys


def per_kernel(root, prefix, name):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{root}/{prefix}_{name}/**/*counter_collection.csv", recursive=True):
        per_disp = collections.defaultdict(float)
        key_of = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            d = r["Dispatch_Id"]
            per_disp[d] += float(r["Counter_Value"])
            key_of[d] = (r["Kernel_Name"].split("(")[0][:90], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        for d, v in per_disp.items():
            acc[key_of[d]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(root):
    out = []
    for prefix in ("pmc", "pmcil"):
        fetch, write = per_kernel(root, prefix, "FETCH_SIZE"), per_kernel(root, prefix, "WRITE_SIZE")
        for k in sorted(set(fetch) & set(write)):
            out.append({"kernel": k[0], "grid": k[1], "fetch_kb": round(fetch[k], 1),
                        "write_kb": round(write[k], 1),
                        "hbm_bytes": round((2 * fetch[k] + write[k]) * 1024)})
    rows = [json.loads(l) for l in open(f"{root}/rows.jsonl") if l.startswith("{")]
    res = {"traffic_per_dispatch": out, "rows_bench": rows,
           "note": "traffic = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (KB x 1024); rows_bench = "
                   "tools/bench_rows.py (HIP-event us, algorithmic bytes, HBM fraction)"}
    with open(f"{root}/traffic.json", "w") as f:
        json.dump(res, f, indent=1)
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main(sys.argv[1])
