#!/bin/bash
# forward 2048 x 1712 x 960 under each abv6 variant (timing diagnostics)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in main abv6/*.so; do
  [ "$so" = main ] && L="" || L="RS_LIB_PATH=$so"
  for f in ${FORMS:-"fwd 2048 1712 960 0"}; do :; done
  echo -n "$(basename $so .so) "
  env $L timeout -k 10 60 python3 tools/gemm_one.py ${ARGS:-fwd 2048 1712 960 0} 2>&1 | grep -v amdgpu || exit 1
done
