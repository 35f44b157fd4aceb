#!/bin/bash
# HBM traffic of the configs 4/5 gather-side kernels (tools/bench_rows.py: DIN fwd/bwd, staytime
# DIN fwd/bwd, sequence lookup) and of the config-3 many-field IL kernels (tools/il_large_bench.py):
# FETCH_SIZE and WRITE_SIZE in separate kernel-trace PMC passes, then tools/pmc_rows_json.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_rows
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_rows.py --reps 20 > $OUT/rows.jsonl 2>$OUT/rows.err || { echo "rows failed"; tail -5 $OUT/rows.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
    python3 tools/bench_rows.py --reps 3 > $OUT/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmcil_$c -o run -- \
    python3 tools/il_large_bench.py > $OUT/pmcil_$c.log 2>&1 || { echo "pmc il $c failed"; tail -5 $OUT/pmcil_$c.log; exit 1; }
done
python3 tools/pmc_rows_json.py $OUT
