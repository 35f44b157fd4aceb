#!/bin/bash
# wide IL at B = 4500 under two forward grids; GEMM shapes of configs 3 / 5 vs torch.mm
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_diag; mkdir -p $D
timeout -k 10 180 python3 -u tools/diag_wide4500.py > $D/diag_4096.log 2>&1 &&
RS_IL_WIDE_FWD_GRID=2048 timeout -k 10 180 python3 -u tools/diag_wide4500.py > $D/diag_2048.log 2>&1 &&
timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload staytime > $D/gemm_staytime.log 2>&1 &&
timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload multi_head > $D/gemm_multi_head.log 2>&1
rc=$?; cat $D/diag_*.log; tail -3 $D/gemm_*.log; exit $rc
