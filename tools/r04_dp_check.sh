#!/bin/bash
# data-parallel tests (2 ranks on one GPU) after the rows-mode DP tail, plus the rows-mode test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_dp.py \
  tests/test_gpu_dp_graph.py tests/test_gpu_rows_mode.py tests/test_gpu_fullsize.py > gpurun_out/r04_final/pytest_dp.log 2>&1
rc=$?; tail -3 gpurun_out/r04_final/pytest_dp.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04_final/pytest_dp.log | head; exit $rc
