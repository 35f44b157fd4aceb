"""Average PMC counters per kernel over rocprofv3 --pmc passes (tools/pmc_il.sh, pmc_bench.sh).
    python tools/pmc_read.py <dir> [all]   ('all': every kernel, else only IL / reduce kernels)"""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
show_all = len(sys.argv) > 2 and sys.argv[2] == "all"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not show_all and "rs_il" not in k and "column" not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k)
    print("   " + "  ".join(f"{c}={m[c]:.0f}" for c in sorted(m)))
    w = m.get("SQ_WAVES")
    if w:
        per = {c: m[c] / w for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                                    "SQ_INSTS_VMEM_WR") if c in m}
        print("   per-wave: " + "  ".join(f"{c[9:]}={v:.0f}" for c, v in per.items()))
    if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
        wc = m["SQ_WAVE_CYCLES"]
        print(f"   wait_any {m['SQ_WAIT_ANY'] / wc:.2f}  wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
              f"  active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}"
              + (f"  wave_cycles/wave {wc / w:.0f}" if w else ""))
