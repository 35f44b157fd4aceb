#!/bin/bash
# the wide forward's persistent grid at B = 4096 / 2048 (resident capacity ~6 workgroups per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_fwdgrid
mkdir -p $D
export TMPDIR=/tmp
for B in 4096 2048; do for g in 2048 1536 1024 4096; do
  RS_IL_WIDE_FWD_GRID=$g timeout -k 10 200 python3 bench.py --global-batch $B --steps 200 --warmup 20 --no-cpu-baseline --no-bf16 > $D/b${B}_g$g.log 2>&1 || exit $?
  grep '^{' $D/b${B}_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B grid=$g', d['ms_per_step'], d['il_fwd_us'])"
done; done
