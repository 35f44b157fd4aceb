#!/bin/bash
# round-4 iteration 5: deferred dW1 (head stores dz1, the tail forms x0^T dz1) parity + timing,
# the standalone sweep's fixed cost, and the B = 512 / 4096 kernel table again
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_head.py \
  tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_dp_graph.py tests/test_gpu_trainer.py \
  tests/test_gpu_parity.py tests/test_gpu_deterministic.py tests/test_gpu_golden.py tests/test_gpu_dp.py tests/test_gpu_export.py tests/test_gpu_metrics.py > gpurun_out/pt5.log 2>&1
rc=$?; tail -2 gpurun_out/pt5.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt5.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 tools/sweep_bench.py > gpurun_out/sweep5.log 2>&1 || exit $?
cat gpurun_out/sweep5.log
for v in 0 1; do
  RS_HEAD_W1_PARTIALS=$([ $v = 1 ] && echo 1) timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 \
    --no-cpu-baseline --no-bf16 > gpurun_out/ab5_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab5_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w1partials=$v', d['ms_per_step'], d['roofline']['launch_us'])"
done
BATCHES="512 4096" OUT=gpurun_out/r04_dz bash tools/small_batch.sh
