#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (separate from PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_NAME:-prof}
timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline --kernel-reps 20 \
  > gpurun_out/${PROF_NAME:-prof}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${PROF_NAME:-prof}_bench.log
find $OUT -name "*stats*" | head; exit $rc
