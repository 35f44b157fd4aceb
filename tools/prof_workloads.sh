#!/bin/bash
# Timed-steps-only kernel breakdown of configs 3-5 (and config 2): rocprofv3 kernel trace of
# bench.py --trace-markers, cut to the timed loop by tools/prof_steps.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/steps}
mkdir -p $D
export TMPDIR=/tmp
for w in ${WORKLOADS:-multi_head din staytime autoint}; do
  extra=""; [ $w = autoint ] && extra="--no-bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/$w -o run -- python3 bench.py --workload $w --steps 20 --warmup 5 --trace-markers --no-cpu-baseline --kernel-reps 2 $extra > $D/$w.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$w rc=$rc"; tail -5 $D/$w.log; exit $rc; }
  grep '^{' $D/$w.log | cut -c1-200
  python3 tools/prof_steps.py $D/$w 20 0 $D/$w.json | head -30
done
