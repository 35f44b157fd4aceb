#!/bin/bash
# branch-free scalar loads for unaligned GEMM operands: GEMM parity, full suite, configs 3 / 5 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_scalar; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
for w in multi_head staytime; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_$w.log 2>&1 || exit 1
  echo "$w $(grep '^{' $D/wl_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload multi_head --min-macs 2.6e8 > $D/gemm_multi_head.log 2>&1 || exit 1
grep kind $D/gemm_multi_head.log
