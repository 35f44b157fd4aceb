#!/bin/bash
# round-4 iteration 9: split-K weight gradients reduced inside the GEMM launch (config 5's
# column_reduce passes), A/B against the separate reduce on the config-5 / config-3 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_it9
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_ops.py \
  tests/test_gpu_towers.py tests/test_gpu_models.py tests/test_gpu_rank_models.py tests/test_gpu_trainer.py \
  tests/test_gpu_dp_graph.py tests/test_gpu_glue.py > $D/pt.log 2>&1
rc=$?; tail -2 $D/pt.log; grep -E "^(FAILED|ERROR)" $D/pt.log | head; [ $rc -le 1 ] || exit $rc
for w in staytime multi_head; do for v in 1 0; do
  RS_GEMM_SPLIT_REDUCE=$v timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $D/${w}_$v.log 2>&1 || exit $?
  grep '^{' $D/${w}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w fused=$v', d['ms_per_step'], d['value'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/st -o run -- python3 bench.py --workload staytime --steps 20 --warmup 5 --no-cpu-baseline --trace-markers --kernel-reps 2 > $D/st_traced.log 2>&1 || exit $?
python3 tools/prof_steps.py $D/st 20 0 $D/staytime.json | head -14
