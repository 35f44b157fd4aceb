#!/bin/bash
# round-4 iteration 6: deferred dW1 with batched loads / prefetched Adam operands / xt blocks first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_il_wide.py tests/test_gpu_dp.py tests/test_gpu_dp_graph.py tests/test_gpu_bf16.py tests/test_gpu_export.py > gpurun_out/pt6.log 2>&1
rc=$?; tail -2 gpurun_out/pt6.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt6.log | head; [ $rc -le 1 ] || exit $rc
for B in 4096 512; do for v in 0 1; do
  RS_HEAD_W1_PARTIALS=$([ $v = 1 ] && echo 1) timeout -k 10 200 python3 bench.py --global-batch $B --steps 200 --warmup 20 \
    --no-cpu-baseline --no-bf16 > gpurun_out/ab6_${B}_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab6_${B}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B w1partials=$v', d['ms_per_step'], d['roofline']['launch_us'])"
done; done
BATCHES="512 4096" OUT=gpurun_out/r04_dz3 bash tools/small_batch.sh
