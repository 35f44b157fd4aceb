#!/bin/bash
# Kernel-only durations of tools/push_bench.py under rocprofv3 (event timing adds launch
# overhead): one kernel-stats table per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/push_prof}
mkdir -p $D
export TMPDIR=/tmp
i=0
for setting in ${SETTINGS:-RS_NONE=0}; do
  i=$((i+1))
  for c in ${CASES:-c3 c4_hist c4_q}; do
    env $setting timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/s$i/$c -o run -- \
      python3 tools/push_bench.py --only $c --reps 10 > $D/s$i.$c.log 2>&1 || { echo "failed $setting $c"; tail -3 $D/s$i.$c.log; exit 1; }
    f=$(find $D/s$i/$c -name "*kernel_stats.csv" | head -1)
    python3 - "$setting" "$c" "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[3])) if "accum" in r["Name"] or "push_" in r["Name"]]
for r in rows:
    print(sys.argv[1], sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg")
PY
  done
done
