#!/bin/bash
# SQ counters of one large-GEMM launch form (tools/gemm_one.py), one pass per counter set
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${D:-gpurun_out/gemm_pmc}; mkdir -p $D; export TMPDIR=/tmp
ARGS=${ARGS:-"fwd 2048 1712 960 0"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE"
k=0
for P in "$P1" "$P2"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $D/p$k -o run -- python3 tools/gemm_one.py $ARGS > $D/p$k.log 2>&1 || { echo "pass $k failed"; tail -5 $D/p$k.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "big_kernel" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(n[k], 1):14.0f}")
PY
