#!/bin/bash
# Same-box A/B of bench.py under environment variants: ab_bench.sh "LABEL:VAR=val ..." ...
# (each variant run REPS times, interleaved; prints label, samples/s, ms/step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in $(seq ${REPS:-2}); do
  for spec in "$@"; do
    label=${spec%%:*}; vars=${spec#*:}
    env $vars timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline \
      --no-bf16 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/ab.log; exit 1; }
    python3 - "$label" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab.log") if l.startswith("{")][0])
print(sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["launch_us"])
PY
  done
done
