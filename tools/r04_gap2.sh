#!/bin/bash
# the 20-step vs 200-step gap: per-step device times (RS_BENCH_STEP_TRACE) with and without the
# capture-time graph priming (RS_NO_GRAPH_PRIME=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/r04_gap2}
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
  for spec in "noprime20:RS_NO_GRAPH_PRIME=1:20:5" "prime20::20:5" "prime200::200:20"; do
    IFS=: read name env steps warm <<< "$spec"
    env RS_BENCH_STEP_TRACE=1 $env timeout -k 10 200 python bench.py --steps $steps --warmup $warm \
      --no-cpu-baseline --no-bf16 > $D/$name.$k.log 2> $D/$name.$k.err || { echo "$name failed"; tail -3 $D/$name.$k.err; exit 1; }
    python3 - $D/$name.$k.log $D/$name.$k.err $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
t = json.loads([l for l in open(sys.argv[2]) if l.startswith('{"step_trace_us"')][0])
us = t["step_trace_us"]
print(sys.argv[3], d["ms_per_step"], "bwd", d["roofline"]["launch_us"], "fwd", d["il_fwd_us"],
      "first8", us[:8], "median", sorted(us)[len(us) // 2], "last4", us[-4:])
PY
  done
done
