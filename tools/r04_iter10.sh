#!/bin/bash
# round-4 iteration 10: the AutoInt head fused into the wide forward for per-GPU batches <= 1536
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_it10
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_head.py tests/test_gpu_il_wide.py tests/test_gpu_parity.py tests/test_gpu_golden.py \
  tests/test_gpu_metrics.py tests/test_gpu_dp.py tests/test_gpu_export.py > $D/pt.log 2>&1
rc=$?; tail -2 $D/pt.log; grep -E "^(FAILED|ERROR)" $D/pt.log | head; [ $rc -le 1 ] || exit $rc
for B in 512 1024 2048; do for mx in 0 4096; do
  RS_HEAD_FUSE_MAXB=$mx timeout -k 10 200 python3 bench.py --global-batch $B --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/b${B}_$mx.log 2>&1 || exit $?
  grep '^{' $D/b${B}_$mx.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B fusemax=$mx', d['ms_per_step'], d['roofline']['launch_us'], d['il_fwd_us'])"
done; done
RS_HEAD_FUSE_MAXB=4096 timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/b4096_fused.log 2>&1 || exit $?
grep '^{' $D/b4096_fused.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=4096 fused', d['ms_per_step'])"
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/b4096_sep.log 2>&1 || exit $?
grep '^{' $D/b4096_sep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=4096 separate', d['ms_per_step'])"
BATCHES="512 1024" OUT=$D/sb bash tools/small_batch.sh
