#!/bin/bash
# large-GEMM blocks: parity, per-shape timings vs torch.mm, configs 3 / 5 step times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_gemm; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py "tests/test_gpu_parity.py::test_dense_fwd_bwd" > $D/pytest.log 2>&1 &&
timeout -k 10 180 python3 -u tools/diag_wide4500.py > $D/diag_4096.log 2>&1 &&
timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload staytime > $D/gemm_staytime.log 2>&1 &&
timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload multi_head > $D/gemm_multi_head.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload staytime --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_staytime.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload multi_head --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_multi_head.log 2>&1 &&
RS_GEMM_TUNE=512,512,1024,128,512,0 timeout -k 10 300 python3 -u bench.py --workload staytime --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_staytime_old.log 2>&1 &&
RS_GEMM_TUNE=512,512,1024,128,512,0 timeout -k 10 300 python3 -u bench.py --workload multi_head --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_multi_head_old.log 2>&1
rc=$?; tail -2 $D/pytest.log; cat $D/diag_4096.log; for f in $D/gemm_*.log; do tail -1 $f; done
for f in $D/wl_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; done; exit $rc
