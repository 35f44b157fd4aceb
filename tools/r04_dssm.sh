#!/bin/bash
# DSSM heads / teacher-student layers grouped: full GPU suite, config-5 step, launches per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_dssm; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --workload staytime --steps 50 --warmup 10 --no-cpu-baseline > $D/wl_staytime_$r.log 2>&1 || exit 1
echo "staytime $(grep '^{' $D/wl_staytime_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/st -o run -- python3 bench.py --workload staytime --steps 20 --warmup 5 --no-cpu-baseline --trace-markers --kernel-reps 2 > $D/st_traced.log 2>&1 || exit 1
python3 tools/prof_steps.py $D/st 20 0 $D/staytime.json | head -3
