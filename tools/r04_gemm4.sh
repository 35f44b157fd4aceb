#!/bin/bash
# GEMM engine (interior slabs: straight-line loads): parity, forced-tile sweep, workload steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/${OUT:-r04_gemm4}; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_il_wide.py "tests/test_gpu_parity.py::test_dense_fwd_bwd" > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
for t in ${TILES:-old 64x64 64x128 128x64 128x128}; do
  for w in staytime multi_head; do
    if [ $t = old ]; then export RS_GEMM_TUNE=512,512,1024,128,512,0; unset RS_GEMM_BIG_TILE; else unset RS_GEMM_TUNE; export RS_GEMM_BIG_TILE=$t; fi
    timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w --min-macs 2.6e8 > $D/${w}_$t.log 2>&1 || exit 1
  done
done
unset RS_GEMM_TUNE RS_GEMM_BIG_TILE
for w in staytime multi_head; do
  timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w > $D/${w}_auto_all.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_$w.json.log 2>&1 || exit 1
  RS_GEMM_TUNE=512,512,1024,128,512,0 timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_${w}_mf16.json.log 2>&1 || exit 1
done
tail -2 $D/pytest.log; for f in $D/wl_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; done; exit 0
