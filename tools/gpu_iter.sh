#!/bin/bash
# Iteration session: GPU tests, IL kernel timing of the in-tree library and of variant libraries
# (VARIANTS="name:path ..."), short bench, 2-rank DP rehearsal on the one GPU, SQ PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; return $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pt.log 2>&1
  echo "pytest rc=$?"; tail -3 gpurun_out/pt.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt.log | head
fi
echo "il base $(step 120 python tools/il_bench.py)"
for v in $VARIANTS; do n=${v%%:*}; p=${v#*:}; echo "il $n $(RS_LIB_PATH=$p step 120 python tools/il_bench.py)"; done
step 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b.log 2>&1; echo "bench rc=$?"; grep '^{' gpurun_out/b.log | cut -c1-400
for v in $VARIANTS; do n=${v%%:*}; p=${v#*:}; RS_LIB_PATH=$p step 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_$n.log 2>&1; echo "bench $n rc=$?"; grep '^{' gpurun_out/b_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['il_fwd_us'])"; done
if [ -n "$DP" ]; then
  step 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 30 --warmup 5 > gpurun_out/b_dp2.log 2>&1; echo "dp2 rc=$?"; grep '^{' gpurun_out/b_dp2.log | cut -c1-300
fi
if [ -n "$PMC" ]; then
  for c in $PMC; do
    REPS=5 step 120 rocprofv3 --kernel-trace --pmc ${c//,/ } --output-format csv -d gpurun_out/pmc_${c%%,*} -o run -- python3 tools/il_bench.py > gpurun_out/pmc_${c%%,*}.log 2>&1; echo "pmc $c rc=$?"
  done
fi
exit 0
