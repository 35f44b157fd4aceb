#!/bin/bash
# tile-group / XCD-remap sweep of the forward 2048 x 1712 x 960 (full kernel and loads only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in main abv6/nomfma.so; do
  [ "$so" = main ] && L="" || L="RS_LIB_PATH=$so"
  for gm in 0 1 2 4 8 16; do
    echo -n "$(basename $so .so) gm=$gm "
    env $L RS_GEMM_BIG_GM=$gm timeout -k 10 60 python3 tools/gemm_one.py fwd 2048 1712 960 0 2>&1 | grep -v amdgpu || exit 1
  done
done
