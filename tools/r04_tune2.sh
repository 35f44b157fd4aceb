#!/bin/bash
# second split / tile policy sweep (big_min, narrow_below lowered)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_tune2; mkdir -p $D
for tune in "256,512,1024,128,256" "128,512,1024,128,128" "256,512,1024,128,128" "128,512,1024,128,256" "256,512,512,128,256" "256,256,1024,128,256" "64,512,1024,128,64"; do
  for w in staytime multi_head din; do
    RS_GEMM_TUNE=$tune timeout -k 10 240 python3 bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline \
      > $D/${w}_${tune//,/_}.log 2>&1 || { echo "failed $w $tune"; exit 1; }
    echo "$tune $w $(grep '^{' $D/${w}_${tune//,/_}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
