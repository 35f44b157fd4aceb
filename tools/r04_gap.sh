#!/bin/bash
# Driver-exact bench (--steps 20 --warmup 5) and a 200-step run back to back on one box, twice
# interleaved, then the per-GPU-batch table (tools/small_batch.sh).  VERDICT r03 item 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/r04_gap}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/drv_full.log 2>&1 || exit $?
grep '^{' $D/drv_full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('drv_full', d['value'], d['ms_per_step'], d['roofline']['frac'], d['bf16']['value'])"
for k in 1 2; do
  for st in "20 5" "200 20"; do
    set -- $st
    timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-bf16 > $D/s$1_$k.log 2>&1 || exit $?
    grep '^{' $D/s$1_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps', $1, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launch_us'], d['il_fwd_us'])"
  done
done
[ -n "$NO_SB" ] || OUT=$D/sb bash tools/small_batch.sh
