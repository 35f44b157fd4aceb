#!/bin/bash
# after the forward grid change: IL / full-size parity, the default and driver-length bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final_d
mkdir -p $D
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_il_wide.py \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_bf16.py > $D/pt.log 2>&1
rc=$?; tail -2 $D/pt.log; grep -E "^(FAILED|ERROR)" $D/pt.log | head; [ $rc -eq 0 ] || exit $rc
step 300 python3 bench.py > $D/bench_default.log 2>&1
grep '^{' $D/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['il_fwd_us'], d['bf16']['value'], d['bf16']['ms_per_step'])"
step 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_20_5.log 2>&1
grep '^{' $D/bench_20_5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('20/5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
BATCHES="4096" OUT=$D/sb bash tools/small_batch.sh
