#!/bin/bash
# forced tile / split sweep of the big GEMM kernels over the configs 3 / 5 trunk shapes
# (RS_GEMM_BIG_TILE=BMxBN,S; HIP events, tools/gemm_one.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shape in "4096 1616 273 0" "2048 1712 960 1" "2048 1840 400 0"; do
  for form in ${FORMS:-fwd weight data}; do
    echo -n "auto "; timeout -k 10 60 python3 tools/gemm_one.py $form $shape 2>&1 | grep -v amdgpu || exit 1
    for t in ${TILES:-128x128 128x64 64x64}; do
      for s in ${SPLITS:-1 2 4}; do
        echo -n "$t,$s "
        RS_GEMM_BIG_TILE=$t,$s timeout -k 10 60 python3 tools/gemm_one.py $form $shape 2>&1 | grep -v amdgpu || exit 1
      done
    done
  done
done
