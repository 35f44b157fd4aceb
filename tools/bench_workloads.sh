#!/bin/bash
# Configs 3-5 on one GPU (per-GPU batch of the stated DP degree) + rocprofv3 kernel stats of each.
# Usage (GPU box): bash tools/bench_workloads.sh [round-tag]
set -o pipefail
R=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$R
for w in multi_head din staytime; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 > gpurun_out/$R/bench_$w.log 2>&1 || { echo "bench $w failed rc=$?"; tail -20 gpurun_out/$R/bench_$w.log; exit 1; }
  grep '^{' gpurun_out/$R/bench_$w.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof_$w -o prof -- python3 bench.py --workload $w --steps 10 --warmup 3 > gpurun_out/$R/prof_$w.log 2>&1 || { echo "prof $w failed rc=$?"; tail -20 gpurun_out/$R/prof_$w.log; exit 1; }
done
echo done
