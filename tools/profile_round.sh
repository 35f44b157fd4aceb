#!/bin/bash
# Round profile: (1) rocprofv3 kernel trace + stats of the default bench command, (2) separate
# PMC passes (kernel-trace only) for the IL backward's HBM traffic: FETCH_SIZE and WRITE_SIZE in
# their own passes (MI355X_MICROARCH.md: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r01}
mkdir -p gpurun_out/$R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/trace -o run -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --kernel-reps 50 > gpurun_out/$R/bench_traced.log 2>&1 || exit $?
echo traced ok
for c in FETCH_SIZE WRITE_SIZE; do
  IL_BENCH_ONLY=push_hot_base_saved REPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/$R/pmc_$c -o run -- \
    python3 tools/il_bench.py > gpurun_out/$R/pmc_$c.log 2>&1 || exit $?
  echo pmc $c ok
done
