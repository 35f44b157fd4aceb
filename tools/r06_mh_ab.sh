#!/bin/bash
# Config-3 push and step: the counting-sort multi-hot push vs the LDS-atomic CAS push
# (RS_PUSH_MH_CAS=1), kernel-only (tools/push_prof.sh) and bench.py --workload multi_head.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/mh_ab}
mkdir -p $D
OUT=$D/prof SETTINGS="RS_NONE=0 RS_PUSH_MH_CAS=1" CASES="c3 c3_scan" bash tools/push_prof.sh || exit 1
for r in 1 2; do
  for v in sort cas; do
    if [ $v = cas ]; then E="RS_PUSH_MH_CAS=1"; else E="RS_NONE=0"; fi
    env $E timeout -k 10 300 python bench.py --workload multi_head --steps 40 --warmup 10 > $D/mh_${v}_$r.log 2>&1 || { echo "fail $v"; tail -3 $D/mh_${v}_$r.log; exit 1; }
    echo "multi_head $v $r $(python3 -c "import json; d=json.loads(open('$D/mh_${v}_$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
