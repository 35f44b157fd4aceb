#!/bin/bash
# round-4 close: smoke, default bench, config-5 bench line with its CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final_g; mkdir -p $D
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python3 -u bench.py > $D/bench_default.log 2>&1 || exit 1
grep '^{' $D/bench_default.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["roofline"]["frac"])'
for w in staytime multi_head; do
  timeout -k 10 300 python3 -u bench.py --workload $w > $D/wl_$w.log 2>&1 || exit 1
  echo "$w $(grep '^{' $D/wl_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
