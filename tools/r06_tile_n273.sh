#!/bin/bash
# forced tiles for the N = 273 trunk forward / weight products (config 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for form in fwd weight; do
  echo -n "auto "; timeout -k 10 60 python3 tools/gemm_one.py $form 4096 1616 273 0 2>&1 | grep -v amdgpu || exit 1
  for t in 128x32,1 128x32,2 128x32,4 128x32,8 64x64,8 64x64,16 128x64,8; do
    echo -n "$t "; RS_GEMM_BIG_TILE=$t timeout -k 10 60 python3 tools/gemm_one.py $form 4096 1616 273 0 2>&1 | grep -v amdgpu || exit 1
  done
done
