#!/bin/bash
# large-GEMM block sweep (forced tiles) on the configs 3 / 5 large shapes; IL wide diagnostic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_gemm2; mkdir -p $D
timeout -k 10 300 python3 -u tools/diag_wide4500b.py > $D/diag_b.log 2>&1 || echo "diag failed"
for t in 64x64 64x128 128x64 128x128; do
  for w in staytime multi_head; do
    RS_GEMM_BIG_TILE=$t timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w --min-macs 2.6e8 > $D/${w}_$t.log 2>&1 || exit 1
  done
done
for w in staytime multi_head; do
  RS_GEMM_TUNE=512,512,1024,128,512,0 timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w --min-macs 2.6e8 > $D/${w}_old.log 2>&1 || exit 1
done
cat $D/diag_b.log; grep -h '"kind"' $D/*.log | sort > $D/all.txt; exit 0
