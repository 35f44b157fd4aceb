#!/bin/bash
# PMC evidence for the dominant kernels, each counter set in its own kernel-trace-only pass:
#   IL backward v4 + fused push (tools/il_bench.py): FETCH_SIZE, WRITE_SIZE (the bench line's
#   traffic comes from tools/measure.sh pmc over bench.py itself);
#   its SQ counters (tools/pmc_il_sq.sh groups); the config-4 history push (tools/push_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/pmc}
mkdir -p $D
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  IL_BENCH_ONLY=push_hot_base_saved REPS=10 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/pmc_$c -o run -- \
    python3 tools/il_bench.py > $D/pmc_$c.log 2>&1 || { echo "il pmc $c failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/push_$c -o run -- \
    python3 tools/push_bench.py --only c4_hist,c3 --reps 5 > $D/push_$c.log 2>&1 || { echo "push pmc $c failed"; exit 1; }
done
PMC_DIR=$D/sq bash tools/pmc_il_sq.sh > $D/sq.txt 2>&1; rc=$?; tail -30 $D/sq.txt; exit $rc
