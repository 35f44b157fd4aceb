#!/bin/bash
# quick iteration: wide-kernel parity, the elimination timings, and the A/B at two batches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/r04_iter}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_il_wide.py tests/test_gpu_metrics.py tests/test_gpu_dp_graph.py ${EXTRA_TESTS} > $D/pytest.log 2>&1
rc=$?; tail -2 $D/pytest.log; grep -E "^(FAILED|ERROR)" $D/pytest.log | head -10; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/il_variants.py > $D/ilvar.txt 2>&1 || exit $?
cat $D/ilvar.txt | grep -v amdgpu.ids
for gb in ${BATCHES:-512 1024 2048}; do
  for v in ${VARIANTS:-wave wide}; do
    RS_IL_VARIANT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --global-batch $gb \
      --no-cpu-baseline --no-bf16 > $D/ab.log 2>&1 || { echo "$v $gb failed"; tail -5 $D/ab.log; exit 1; }
    grep '^{' $D/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $gb, d['value'], d['ms_per_step'], 'bwd', d['roofline']['launch_us'], 'fwd', d['il_fwd_us'])"
  done
done
# the head's phase cycles (block 0, s_memtime; diagnostic build in _gpuvar/)
if [ -f _gpuvar/librecsys_hstamps.so ]; then
  HEAD_STAMPS=1 RS_LIB_PATH=_gpuvar/librecsys_hstamps.so timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'tools'); sys.path.insert(0, '.')
import head_bench as hb
for B in (512, 4096):
    us, st = hb.bench(B, reps=50)
    print('head stamps B', B, us, 'us (stamped build); phases (cycles):', st)
" 2>&1 | grep -v amdgpu.ids
fi
# driver-exact bench vs a 200-step run, back to back
[ -n "$NO_GAP" ] || NO_SB=1 OUT=$D/gap bash tools/r04_gap.sh
