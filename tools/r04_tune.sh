#!/bin/bash
# split-K policy sweep after the GEMM slab-pipeline change: configs 3 / 5 steps per RS_GEMM_TUNE
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_tune; mkdir -p $D
for tune in "512,512,1024,128,512" "512,256,1024,128,512" "512,512,512,128,512" "512,512,1024,256,512" "512,128,512,256,512" "512,512,2048,128,512" "256,512,1024,128,256"; do
  for w in staytime multi_head; do
    RS_GEMM_TUNE=$tune timeout -k 10 240 python3 bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline \
      > $D/${w}_${tune//,/_}.log 2>&1 || { echo "failed $w $tune"; exit 1; }
    echo "$tune $w $(grep '^{' $D/${w}_${tune//,/_}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
