#!/bin/bash
# PMC passes (kernel-trace only, one counter group per pass) over a short default bench run:
# per-kernel wave/wait/instruction counters for every kernel of the step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PMC_OUT:-pmcb}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-reps 2 ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_read.py $OUT all
