#!/bin/bash
# the big GEMM kernels' plans on every configs 3 / 5 product (default threshold 2^29 multiply-adds,
# and with the big kernels from 2^26), then the two workloads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${1:-gpurun_out/plan}; mkdir -p $D
for w in multi_head staytime; do
  timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${w}_big.jsonl 2>&1 || { tail -5 $D/${w}_big.jsonl; exit 1; }
  RS_GEMM_BIG_MACS=67108864 timeout -k 10 200 python3 tools/gemm_shapes.py --workload $w --min-macs 1e7 > $D/${w}_big26.jsonl 2>&1 || exit 1
done
python3 - $D <<'PY'
import json, sys
d = sys.argv[1]
for w in ("multi_head", "staytime"):
    big = [json.loads(l) for l in open(f"{d}/{w}_big.jsonl") if l.startswith("{")]
    b26 = [json.loads(l) for l in open(f"{d}/{w}_big26.jsonl") if l.startswith("{")]
    e = {(r["kind"], r["M"], r["K"], r["N"], r["act"]): r for r in b26 if "kind" in r}
    for r in big:
        if "kind" not in r:
            print(w, "TOTAL", r["gemm_us_per_step"], "blas", r["blas_us_per_step"]); continue
        k = (r["kind"], r["M"], r["K"], r["N"], r["act"])
        print(w, *k, "x", r["calls"], "us", r["us"], "from2^26", e[k]["us"] if k in e else None, "blas", r["blas_us"])
    for r in b26:
        if "kind" not in r: print(w, "TOTAL from2^26", r["gemm_us_per_step"])
PY
for w in ${WL:-multi_head staytime}; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_$w.log 2>&1 || exit 1
  grep '^{' $D/wl_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$w', d['value'], d['ms_per_step'])"
done
