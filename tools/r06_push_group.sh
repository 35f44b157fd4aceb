cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/grp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "grouped or election or sparse_push" -x -q --timeout 120 --timeout-method thread > gpurun_out/grp/pytest_push.log 2>&1 || { tail -30 gpurun_out/grp/pytest_push.log; exit 1; }
tail -2 gpurun_out/grp/pytest_push.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_models.py tests/test_gpu_trainer.py tests/test_gpu_towers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/grp/pytest_models.log 2>&1 || { tail -30 gpurun_out/grp/pytest_models.log; exit 1; }
tail -2 gpurun_out/grp/pytest_models.log
for k in 1 2; do
for v in 1 0; do
  RS_PUSH_GROUP=$v timeout -k 10 300 python3 bench.py --workload staytime --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/grp/wl_st_$v.log 2>&1 || { tail -5 gpurun_out/grp/wl_st_$v.log; exit 1; }
  grep '^{' gpurun_out/grp/wl_st_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('group=$v', d['value'], d['ms_per_step'])"
done
done
