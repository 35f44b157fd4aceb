#!/bin/bash
# config 3's table in list mode (claims + touched list + list Adam) vs scan mode (flag sweep)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mhscan
for k in 1 2; do
for v in 0 1; do
  RS_MH_SCAN=$v timeout -k 10 300 python3 bench.py --workload multi_head --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/mhscan/wl_$v.log 2>&1 || { tail -5 gpurun_out/mhscan/wl_$v.log; exit 1; }
  grep '^{' gpurun_out/mhscan/wl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('scan=$v', d['value'], d['ms_per_step'])"
done
done
