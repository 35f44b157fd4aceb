#!/bin/bash
# GEMM engine (untransposed LDS for the x-contiguous operands): parity, forced-tile sweep on the
# configs 3 / 5 large shapes, plus the sample-2272 conditioning diagnostic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_gemm3; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py "tests/test_gpu_parity.py::test_dense_fwd_bwd" > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
timeout -k 10 120 python3 -u tools/diag_wide2272.py > $D/diag_2272.log 2>&1 || echo "diag failed"
for t in old 64x64 64x128 128x64 128x128; do
  for w in staytime multi_head; do
    if [ $t = old ]; then export RS_GEMM_TUNE=512,512,1024,128,512,0; unset RS_GEMM_BIG_TILE; else unset RS_GEMM_TUNE; export RS_GEMM_BIG_TILE=$t; fi
    timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w --min-macs 2.6e8 > $D/${w}_$t.log 2>&1 || exit 1
  done
done
unset RS_GEMM_TUNE RS_GEMM_BIG_TILE
for w in staytime multi_head; do
  timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w > $D/${w}_auto_all.log 2>&1 || exit 1
done
tail -2 $D/pytest.log; cat $D/diag_2272.log; exit 0
