#!/bin/bash
# per-shape GEMM times of the configs 3 / 5 steps: big kernels (default) vs the round-4 engine
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${D:-gpurun_out/shapes}; mkdir -p $D
for w in multi_head staytime; do
  timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${w}_big.jsonl 2>&1 || { tail -5 $D/${w}_big.jsonl; exit 1; }
  RS_GEMM_BIG=0 timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${w}_engine.jsonl 2>&1 || exit 1
done
python3 - $D <<'PY'
import json, sys, glob
d = sys.argv[1]
for w in ("multi_head", "staytime"):
    big = [json.loads(l) for l in open(f"{d}/{w}_big.jsonl") if l.startswith("{")]
    eng = [json.loads(l) for l in open(f"{d}/{w}_engine.jsonl") if l.startswith("{")]
    e = {(r["kind"], r["M"], r["K"], r["N"], r["act"]): r for r in eng if "kind" in r}
    for r in big:
        if "kind" not in r:
            print(w, "TOTAL big", r["gemm_us_per_step"], "blas", r["blas_us_per_step"]); continue
        k = (r["kind"], r["M"], r["K"], r["N"], r["act"])
        print(w, *k, "x", r["calls"], "big", r["us"], "engine", e[k]["us"] if k in e else None, "blas", r["blas_us"])
    for r in eng:
        if "kind" not in r: print(w, "TOTAL engine", r["gemm_us_per_step"])
PY
