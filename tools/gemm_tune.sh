#!/bin/bash
# GEMM tile/split policy sweep on the GPU box: the configs 3 and 5 workload steps under several
# RS_GEMM_TUNE settings (big_min, split_below, split_target, min_rows; dense.hip::gemm_tune).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gemm_tune
for tune in ${TUNES:-"512,512,1024,128,0" "512,512,1024,128,512" "512,512,1024,128,1024" "1024,512,1024,128,1024"}; do
  for w in ${WORKLOADS:-multi_head staytime}; do
    RS_GEMM_TUNE=$tune timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/gemm_tune/${w}_${tune//,/_}.log 2>&1 || { echo "failed $w $tune"; exit 1; }
    echo "$tune $w $(grep '^{' gpurun_out/gemm_tune/${w}_${tune//,/_}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
