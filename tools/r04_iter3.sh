#!/bin/bash
# round-4 iteration 3: gap diagnosis + the per-GPU-batch kernel table (B = 512 / 1024 / 2048 /
# 4096) + the DP / trainer GPU tests touched by the priming
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_dp_graph.py \
  tests/test_gpu_dp.py tests/test_gpu_trainer.py tests/test_gpu_fullsize.py > gpurun_out/pt3.log 2>&1
rc=$?; tail -2 gpurun_out/pt3.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt3.log | head; [ $rc -le 1 ] || exit $rc
bash tools/r04_gap2.sh || exit $?
OUT=gpurun_out/r04_sb bash tools/small_batch.sh
