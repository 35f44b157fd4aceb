#!/bin/bash
# Config-5 / config-4 steps with the single-hot push's two aggregation forms (RS_PUSH_LDS_ADD=1:
# LDS float atomics; default: counting sort for rows >= 32 floats), two rounds each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/push_ab}
mkdir -p $D
for r in 1 2; do
  for v in sort lds; do
    if [ $v = lds ]; then E="RS_PUSH_LDS_ADD=1"; else E="RS_NONE=0"; fi
    for w in staytime din; do
      env $E timeout -k 10 300 python bench.py --workload $w --steps 40 --warmup 10 > $D/${w}_${v}_$r.log 2>&1 || { echo "fail $w $v"; tail -3 $D/${w}_${v}_$r.log; exit 1; }
      echo "$w $v $r $(python3 -c "import json,sys; d=json.loads(open('$D/${w}_${v}_$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
