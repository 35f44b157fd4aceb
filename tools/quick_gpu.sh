#!/bin/bash
# Iteration loop on the GPU box: full GPU test suite, short bench, kernel-stats profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pt.log 2>&1
rc=$?; tail -4 gpurun_out/pt.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b.log 2>&1
rc=$?; grep '^{' gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d['il_fwd_us'], d['roofline']['launch_us'])"; [ $rc -eq 0 ] || exit $rc
PROF_NAME=prof_q STEPS=30 timeout -k 10 300 bash tools/profile.sh > /dev/null 2>&1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_q/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.2f}")
PY
