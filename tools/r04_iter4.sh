#!/bin/bash
# round-4 iteration 4: head restructure (logits backward folded into the row waves) parity +
# timing, and the optimizer-tail split (RS_NO_FUSED_TAIL: reduction and sweep as two launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_models.py > gpurun_out/pt4.log 2>&1
rc=$?; tail -2 gpurun_out/pt4.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt4.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 tools/head_bench.py > gpurun_out/head4.log 2>&1 || exit $?
cat gpurun_out/head4.log
RS_NO_FUSED_TAIL=1 BATCHES="512 4096" OUT=gpurun_out/r04_tail bash tools/small_batch.sh
