#!/bin/bash
# layer-aligned Trainer arena (+ one-launch Dense backward): full GPU suite, configs 3-5 steps,
# config-5 per-step kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_align; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
for w in staytime multi_head din; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_$w.log 2>&1 || exit 1
  echo "$w $(grep '^{' $D/wl_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/st -o run -- python3 bench.py --workload staytime --steps 20 --warmup 5 --no-cpu-baseline --trace-markers --kernel-reps 2 > $D/st_traced.log 2>&1 || exit 1
python3 tools/prof_steps.py $D/st 20 0 $D/staytime.json > $D/steps.txt; head -3 $D/steps.txt
