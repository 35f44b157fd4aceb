#!/bin/bash
# same-box A/B of GEMM engine builds (_abvar/lib_*.so): per-shape times and workload steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/${OUT:-r04_gemm_ab}; mkdir -p $D
for rep in 1 2; do
for v in ${VARIANTS:-p1i p1m p2m}; do
  export RS_LIB_PATH=$PWD/_abvar/lib_$v.so RS_GEMM_TUNE=512,512,1024,128,512,0
  for w in staytime multi_head; do
    timeout -k 10 240 python3 -u tools/gemm_shapes.py --workload $w --min-macs 1e8 > $D/${w}_${v}_$rep.log 2>&1 || exit 1
  done
  timeout -k 10 300 python3 -u bench.py --workload staytime --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_staytime_${v}_$rep.log 2>&1 || exit 1
  echo "$v $rep $(grep '^{' $D/wl_staytime_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
exit 0
