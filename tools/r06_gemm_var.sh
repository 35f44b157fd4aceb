#!/bin/bash
# per-shape GEMM times (tools/gemm_shapes.py) of the configs 3 / 5 steps under each abv6/*.so
# kernel variant, beside the in-tree library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${1:-gpurun_out/gvar}; mkdir -p $D
for so in main abv6/*.so; do
  n=$(basename $so .so)
  for w in multi_head staytime; do
    if [ "$so" = main ]; then
      timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${n}_$w.jsonl 2>&1 || exit 1
    else
      RS_LIB_PATH=$so timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${n}_$w.jsonl 2>&1 || exit 1
    fi
  done
done
python3 - $D <<'PY'
import json, sys, glob, os
d = sys.argv[1]
res = {}
for f in sorted(glob.glob(f"{d}/*.jsonl")):
    n = os.path.basename(f)[:-6]
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            k = (r["kind"], r["M"], r["K"], r["N"]) if "kind" in r else ("TOTAL",)
            res.setdefault(k, {})[n] = r.get("us", r.get("gemm_us_per_step"))
for k, v in res.items():
    print(*k, " ".join(f"{n}={u}" for n, u in sorted(v.items())))
PY
