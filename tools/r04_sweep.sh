#!/bin/bash
# kernel durations of the scan sweep alone: table size x marked rows (rocprofv3 kernel trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_sweep
export TMPDIR=/tmp
for cfg in "2600000 0" "2600000 5000" "2600000 25000" "260000 0" "260000 5000" "26000 0"; do
  set -- $cfg
  d=gpurun_out/r04_sweep/r$1_k$2
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 tools/sweep_bench.py $1 $2 50 > $d.log 2>&1 || { echo "fail $cfg"; tail -5 $d.log; exit 1; }
  python3 - "$d" "$cfg" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "scan_opt" in r["Name"] or "fill" in r["Name"].lower():
        print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
