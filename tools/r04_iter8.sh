#!/bin/bash
# round-4 iteration 8: bwd4 stages the next iteration's input / the next sample's dy through
# registers (issued after P1 instead of after the K-pass): parity, kernel time, stamps, step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_it8
export TMPDIR=/tmp
D=gpurun_out/r04_it8
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_il_wide.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_deterministic.py \
  tests/test_gpu_head.py tests/test_gpu_bf16.py > $D/pt.log 2>&1
rc=$?; tail -2 $D/pt.log; grep -E "^(FAILED|ERROR)" $D/pt.log | head; [ $rc -le 1 ] || exit $rc
IL_BENCH_ONLY=push_hot_base_saved timeout -k 10 120 python3 tools/il_bench.py > $D/il_bench.txt 2>&1 || exit $?
cat $D/il_bench.txt | tail -1
RS_LIB_PATH=_gpuvar/librecsys_stamps.so timeout -k 10 120 python3 tools/il_stamps.py > $D/stamps.txt 2>&1 || exit $?
cat $D/stamps.txt | tail -10
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/b200_$r.log 2>&1 || exit $?
  grep '^{' $D/b200_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b200', d['ms_per_step'], d['roofline']['launch_us'], d['roofline']['frac'], d['il_fwd_us'])"
done
