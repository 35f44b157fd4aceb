#!/bin/bash
# Same-box GEMM variant timings: tools/gemm_vs_blas.py over the in-tree library and abv6/*.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${D:-gpurun_out/gemm_ab}; mkdir -p $D
[ -n "$TESTS" ] && { timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1; rc=$?; tail -3 $D/pytest.log; [ $rc -ne 0 ] && exit $rc; }
for so in main abv6/*.so; do
  [ "$so" = main ] && L="" || L="RS_LIB_PATH=$so"
  n=$(basename $so .so)
  env $L timeout -k 10 200 python3 tools/gemm_vs_blas.py > $D/gemm_$n.log 2>&1 || { echo "$n failed"; tail -5 $D/gemm_$n.log; exit 1; }
  echo "== $n"; grep -v amdgpu $D/gemm_$n.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['M'],d['K'],d['N'],'fwd',d['fwd_us'],d['blas_fwd_us'],'w',d['wgrad_us'],d['blas_wgrad_us'],'d',d['dgrad_us'],d['blas_dgrad_us'])"
done
