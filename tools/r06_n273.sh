#!/bin/bash
# 128 x 32 tiles for config 3's N = 273 trunk: big-route parity, per-product times, config 3 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/n273
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -k "big_route or large_gemm or split_k" tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/n273/pytest.log 2>&1 || { tail -30 gpurun_out/n273/pytest.log; exit 1; }
tail -2 gpurun_out/n273/pytest.log
for f in fwd weight data; do timeout -k 10 60 python3 tools/gemm_one.py $f 4096 1616 273 0 2>&1 | grep -v amdgpu || exit 1; done
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --workload multi_head --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/n273/wl.log 2>&1 || { tail -5 gpurun_out/n273/wl.log; exit 1; }
  grep '^{' gpurun_out/n273/wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('multi_head', d['value'], d['ms_per_step'])"
done
