import csv, glob, collections, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "rs_il" not in k and "column" not in k:
        continue
    print(k)
    m = {c: sum(v) / len(v) for c, v in d.items()}
    for c in sorted(m):
        print(f"   {c:24s} {m[c]:16.0f}")
    if "SQ_WAVES" in m and "SQ_INSTS_VALU" in m:
        w = m["SQ_WAVES"]
        print(f"   per-wave: VALU {m['SQ_INSTS_VALU']/w:.0f}  LDS {m['SQ_INSTS_LDS']/w:.0f}  SALU {m['SQ_INSTS_SALU']/w:.0f}")
    if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
        print(f"   wait_any/wave_cycles {m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES']:.2f}  active_valu/wave_cycles {m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES']:.2f} lds_bank_conf/active_lds {m['SQ_LDS_BANK_CONFLICT']/max(1,m['SQ_ACTIVE_INST_LDS']):.2f}")
