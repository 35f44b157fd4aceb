#!/bin/bash
# the 2^25 forward threshold / narrow tile order: parity of the big route, the towers' tests,
# config 5 and config 3 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fwd25
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -k "big_route or large_gemm" tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fwd25/pytest.log 2>&1 || { tail -30 gpurun_out/fwd25/pytest.log; exit 1; }
tail -2 gpurun_out/fwd25/pytest.log
for k in 1 2; do
for w in staytime multi_head; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/fwd25/wl_$w.log 2>&1 || { tail -5 gpurun_out/fwd25/wl_$w.log; exit 1; }
  grep '^{' gpurun_out/fwd25/wl_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$w', d['value'], d['ms_per_step'])"
done
done
