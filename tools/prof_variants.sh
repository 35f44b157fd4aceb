#!/bin/bash
# Kernel-stats profile of the bench for the in-tree library and each variant library
# (VARIANTS="name:path ..."), one rocprofv3 kernel-trace pass each; prints the top kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base: $VARIANTS; do
  n=${v%%:*}; p=${v#*:}
  RS_LIB_PATH=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv_$n -o run -- \
    python3 bench.py --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --kernel-reps 10 > gpurun_out/pv_$n.log 2>&1 || exit $?
  echo "== $n $(grep '^{' gpurun_out/pv_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  python3 - $n <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/pv_{sys.argv[1]}/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:7]:
    print(f"  {r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.2f}")
PY
done
