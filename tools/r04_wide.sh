#!/bin/bash
# Wide (4-wave-per-sample) InteractingLayer kernels: parity, then same-box A/B against the
# one-wave-per-sample kernels at per-GPU batch 4096 and 512, then the per-GPU-batch table.
# Plain test failures (rc 1) do not stop the script; faults / timeouts (rc >= 124) do.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/r04_wide}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_il_wide.py tests/test_gpu_metrics.py tests/test_gpu_export.py tests/test_gpu_models.py \
  tests/test_gpu_golden.py tests/test_gpu_fullsize.py \
  "tests/test_gpu_parity.py::test_interacting_small_saved_pair" \
  "tests/test_gpu_parity.py::test_interacting_forward" "tests/test_gpu_parity.py::test_interacting_backward" \
  "tests/test_gpu_parity.py::test_autoint_train_steps_match_oracle" tests/test_gpu_bf16.py > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log; grep -E "^(FAILED|ERROR)" $D/pytest.log | head -20; [ $rc -le 1 ] || exit $rc
for gb in ${BATCHES:-4096 512}; do
  for k in 1 2; do
    for v in wave wide; do
      RS_IL_VARIANT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --global-batch $gb \
        --no-cpu-baseline --no-bf16 > $D/ab.log 2>&1 || { echo "$v $gb failed"; tail -5 $D/ab.log; exit 1; }
      grep '^{' $D/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $gb, d['value'], d['ms_per_step'], 'bwd', d['roofline']['launch_us'], d['roofline']['frac'], 'fwd', d['il_fwd_us'])"
    done
  done
done
[ -n "$NO_SB" ] || OUT=$D/sb bash tools/small_batch.sh
