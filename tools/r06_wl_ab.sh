#!/bin/bash
# configs 3 / 5 step time under the GEMM routes: big kernels (default), the round-4 engine only,
# hipBLASLt (RS_GEMM_BLAS=1); REPS interleaved runs of STEPS steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${D:-gpurun_out/wl_ab}; mkdir -p $D
for k in $(seq ${REPS:-1}); do
for w in ${WLS:-multi_head staytime}; do
  for spec in "big:X=1" "engine:RS_GEMM_BIG=0" "lib:RS_GEMM_BLAS=1"; do
    label=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-40} --warmup 10 --no-cpu-baseline > $D/${w}_$label.log 2>&1 || { echo "$w $label failed"; tail -5 $D/${w}_$label.log; exit 1; }
    python3 - "$w" "$label" "$D/${w}_$label.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"])
PY
  done
done
done
