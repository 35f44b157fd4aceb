#!/bin/bash
# SQ PMC passes (kernel-trace only) over the IL microbenchmark: where the IL waves spend cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${PMC_DIR:-gpurun_out/pmcsq}
mkdir -p $D
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" ; do
  i=$((i+1))
  IL_BENCH_ONLY=${IL_BENCH_ONLY:-push_hot_base_saved} REPS=5 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $D/p$i -o run -- python3 tools/il_bench.py > $D/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_read.py $D
