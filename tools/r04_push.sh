#!/bin/bash
# multi-hot push LDS budget (tile size) A/B at config 3's shape, plus the IL backward alone
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_push
export TMPDIR=/tmp
D=gpurun_out/r04_push
IL_BENCH_ONLY=push_hot_base_saved timeout -k 10 120 python3 tools/il_bench.py > $D/il_bench.txt 2>&1 || exit $?
tail -1 $D/il_bench.txt
for kb in 64 100 150; do
  RS_PUSH_MH_LDS_KB=$kb timeout -k 10 120 python3 tools/push_bench.py --only c3 > $D/c3_$kb.txt 2>&1 || exit $?
  echo "kb=$kb $(tail -1 $D/c3_$kb.txt)"
done
