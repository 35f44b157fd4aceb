#!/bin/bash
# the trunk shapes' three products under each abv6 variant (tools/gemm_one.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
[ -n "$TESTS" ] && { timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/gemm_ab2_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/gemm_ab2_pytest.log; [ $rc -ne 0 ] && exit $rc; }
for so in main abv6/*.so; do
  [ "$so" = main ] && L="" || L="RS_LIB_PATH=$so"
  for f in "fwd 2048 1712 960 1" "weight 2048 1712 960 1" "data 2048 1712 960 1" "fwd 4096 1616 273 0" "weight 4096 1616 273 0" "data 4096 1616 273 0" "fwd 2048 1840 400 0" "weight 2048 1840 400 0"; do
    echo -n "$(basename $so .so) "
    env $L timeout -k 10 60 python3 tools/gemm_one.py $f 2>&1 | grep -v amdgpu || exit 1
  done
done
for f in "fwd 2048 1712 960 1" "weight 2048 1712 960 1" "data 2048 1712 960 1" "fwd 4096 1616 273 0" "weight 4096 1616 273 0" "data 4096 1616 273 0" "fwd 2048 1840 400 0" "weight 2048 1840 400 0"; do
  echo -n "hipBLASLt "; RS_GEMM_BLAS=1 timeout -k 10 60 python3 tools/gemm_one.py $f 2>&1 | grep -v amdgpu || exit 1
done
