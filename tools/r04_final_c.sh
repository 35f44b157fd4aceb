#!/bin/bash
# round-4 final: rows-mode sparse Adam A/B by per-GPU batch, the per-GPU-batch kernel table, the
# B = 512 bench line, and the configs 3-5 workload lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final
mkdir -p $D/rows_mode
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; }
for B in 512 1024 2048 4096; do for mx in 0 1000000; do
  RS_SPARSE_ROWS_MAXN=$mx step 200 python3 bench.py --global-batch $B --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/rows_mode/b${B}_$mx.log 2>&1
  grep '^{' $D/rows_mode/b${B}_$mx.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B rows_maxn=$mx', d['ms_per_step'])"
done; done
OUT=$D/small_batch bash tools/small_batch.sh || exit $?
step 300 python3 bench.py --global-batch 512 > $D/bench_b512.log 2>&1
grep '^{' $D/bench_b512.log | cut -c1-400
for w in multi_head din staytime; do
  step 400 python3 bench.py --workload $w --steps 20 --warmup 5 > $D/wl_$w.log 2>&1
  grep '^{' $D/wl_$w.log | cut -c1-300
done
