#!/bin/bash
# the big GEMM kernels at their current plans with the loads / MFMAs / barriers knocked out
# (abv6/*.so diagnostic builds: wrong results, timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in main abv6/*.so; do
  for a in "fwd 4096 1616 273 0" "weight 4096 1616 273 0" "fwd 2048 1712 960 1" "weight 2048 1712 960 1" "data 2048 1712 960 0" "fwd 2048 1840 400 0" "weight 2048 1840 400 0"; do
    echo -n "$(basename $so .so) "
    if [ $so = main ]; then timeout -k 10 60 python3 tools/gemm_one.py $a 2>&1 | grep -v amdgpu || exit 1
    else RS_LIB_PATH=$so timeout -k 10 60 python3 tools/gemm_one.py $a 2>&1 | grep -v amdgpu || exit 1; fi
  done
done
