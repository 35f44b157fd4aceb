#!/bin/bash
# after the GEMM engine changes: full GPU suite, smoke, default bench, configs 3 / 5 steps (16x16
# blocks vs the opt-in 32x32 blocks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final_e; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python3 -u bench.py > $D/bench_default.log 2>&1 || exit 1
grep '^{' $D/bench_default.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"])'
for w in staytime multi_head din; do
  timeout -k 10 300 python3 -u bench.py --workload $w > $D/wl_$w.log 2>&1 || exit 1
  echo "$w $(grep '^{' $D/wl_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
for w in staytime multi_head; do
  RS_GEMM_TUNE=512,512,1024,128,512,268435456 timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_${w}_mf32.log 2>&1 || exit 1
  echo "$w mf32 $(grep '^{' $D/wl_${w}_mf32.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_${w}_mf16.log 2>&1 || exit 1
  echo "$w mf16 $(grep '^{' $D/wl_${w}_mf16.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
