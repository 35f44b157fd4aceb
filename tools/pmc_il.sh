#!/bin/bash
# PMC passes (kernel-trace only, one counter group per pass) over the IL microbenchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  REPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/il_bench.py > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
