"""Per-step GPU-time breakdown of the TIMED steps only, from a rocprofv3 kernel trace of
`bench.py ... --trace-markers` (the marker kernel 'spin_kernel' is launched right before and right
after the timed loop, outside the timed region).

    python tools/prof_steps.py <trace dir or *_kernel_trace.csv> <steps> [pair index] [out.json]

Prints, per kernel name (shortened), dispatches and microseconds per step, and the split
librecsys_amd kernels / torch kernels / copies+fills; writes the same as JSON when asked.
"""
import csv
import glob
import json
import os
import re
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)                    # drop the argument list
    n = re.sub(r"<.*", "", n) if n.count("<") > 2 else n
    return n[:90]


def origin(name: str) -> str:
    if "copyBuffer" in name or "fillBuffer" in name or "__amd_rocclr" in name:
        return "hip runtime copy/fill"
    if "at::native" in name or "at::" in name or "c10::" in name or "void at" in name:
        return "torch"
    if "nccl" in name.lower() or "rccl" in name.lower():
        return "rccl"
    return "librecsys_amd"


def main(path, steps, pair=0, out=None):
    steps = int(steps)
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    if len(marks) < 2 * (int(pair) + 1):
        raise SystemExit(f"found {len(marks)} marker dispatches; need a pair #{pair}")
    a, b = marks[2 * int(pair)], marks[2 * int(pair) + 1]
    seg = rows[a + 1:b]
    t0 = int(rows[a]["End_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    per = {}
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        e = per.setdefault(k, {"calls": 0, "us": 0.0, "origin": origin(r["Kernel_Name"])})
        e["calls"] += 1
        e["us"] += d
    busy = sum(e["us"] for e in per.values())
    by_origin = {}
    for e in per.values():
        by_origin[e["origin"]] = by_origin.get(e["origin"], 0.0) + e["us"]
    res = {"steps": steps, "wall_us_per_step": round((t1 - t0) / 1e3 / steps, 2),
           "gpu_busy_us_per_step": round(busy / steps, 2),
           "share_by_origin": {k: round(v / busy, 4) for k, v in sorted(by_origin.items())},
           "kernels": sorted(({"name": k, "calls_per_step": round(e["calls"] / steps, 2),
                               "us_per_step": round(e["us"] / steps, 2), "origin": e["origin"],
                               "share": round(e["us"] / busy, 4)} for k, e in per.items()),
                             key=lambda x: -x["us_per_step"])}
    if out:  # written before the listing: a reader that closes the pipe early loses only lines
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    try:
        print(f"wall {res['wall_us_per_step']} us/step, GPU busy {res['gpu_busy_us_per_step']} "
              f"us/step; by origin {res['share_by_origin']}")
        for k in res["kernels"][:40]:
            print(f"  {k['us_per_step']:9.2f} us {k['calls_per_step']:6.1f}x {k['share']*100:5.1f}%  "
                  f"[{k['origin'][:5]}] {k['name']}")
    except BrokenPipeError:
        pass


if __name__ == "__main__":
    main(*sys.argv[1:])
