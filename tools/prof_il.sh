#!/bin/bash
# IL backward evidence: per-phase stamp shares (variant library built with -DRS_IL_STAMPS at
# $STAMPS_LIB), IL kernel timing, and two SQ PMC passes (kernel-trace only) over the bwd variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/il_prof}
mkdir -p $D
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; }
step 120 python tools/il_bench.py > $D/il_bench.txt 2>&1; cat $D/il_bench.txt | tail -3
if [ -n "$STAMPS_LIB" ]; then
  RS_LIB_PATH=$STAMPS_LIB step 120 python tools/il_stamps.py > $D/stamps.txt 2>&1; cat $D/stamps.txt
fi
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  IL_BENCH_ONLY=${ONLY:-bwd} REPS=5 step 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $D/p$i -o run -- python3 tools/il_bench.py > $D/p$i.log 2>&1
done
python3 tools/pmc_read.py $D | tee $D/sq_summary.txt
