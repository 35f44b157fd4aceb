#!/bin/bash
# vectorised list-mode sparse Adam (built, measured no faster, removed in the same round: this is
# the script that produced profiles/r06/push/sparse_adam_vec_ab.txt): whole GPU suite, then config 3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/adamvec
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/adamvec/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/adamvec/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/adamvec/pytest_gpu.log
for k in 1 2; do
for v in vec scalar; do
  if [ $v = scalar ]; then export RS_SPARSE_ADAM_SCALAR=1; else unset RS_SPARSE_ADAM_SCALAR; fi
  timeout -k 10 300 python3 bench.py --workload multi_head --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/adamvec/wl_$v.log 2>&1 || { tail -5 gpurun_out/adamvec/wl_$v.log; exit 1; }
  grep '^{' gpurun_out/adamvec/wl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
done
