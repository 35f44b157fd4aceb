#!/bin/bash
# forced tiles / splits for config 5's 2048 x 1456 x 22 forward (a long reduction, 22 outputs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo -n "auto "; timeout -k 10 60 python3 tools/gemm_one.py fwd 2048 1456 22 1 2>&1 | grep -v amdgpu || exit 1
export RS_GEMM_BIG_MACS=33554432
echo -n "big-auto "; timeout -k 10 60 python3 tools/gemm_one.py fwd 2048 1456 22 1 2>&1 | grep -v amdgpu || exit 1
for t in 64x64,8 64x64,16 64x64,32 128x32,8 128x32,16 128x32,32 128x32,64; do
  echo -n "$t "; RS_GEMM_BIG_TILE=$t timeout -k 10 60 python3 tools/gemm_one.py fwd 2048 1456 22 1 2>&1 | grep -v amdgpu || exit 1
done
unset RS_GEMM_BIG_MACS; echo -n "engine "; RS_GEMM_BIG=0 timeout -k 10 60 python3 tools/gemm_one.py fwd 2048 1456 22 1 2>&1 | grep -v amdgpu || exit 1
