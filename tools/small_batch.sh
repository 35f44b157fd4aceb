#!/bin/bash
# Strong-scaling per-GPU batches on one GPU: the config-2 step at per-GPU batch 512 .. 4096 (what
# ranks of an N = 8 / 4 / 2 / 1 strong-scaling run each process), timed-steps-only kernel
# breakdown from a rocprofv3 kernel trace (tools/prof_steps.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/small_batch}
mkdir -p $D
export TMPDIR=/tmp
for gb in ${BATCHES:-512 1024 2048 4096}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $D/b$gb -o run -- \
    python3 bench.py --global-batch $gb --steps 50 --warmup 10 --trace-markers --no-cpu-baseline \
    --no-bf16 --kernel-reps 20 > $D/b$gb.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "b$gb rc=$rc"; tail -5 $D/b$gb.log; exit $rc; }
  grep '^{' $D/b$gb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B', $gb, d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['il_fwd_us'])"
  python3 tools/prof_steps.py $D/b$gb 50 0 $D/b$gb.json | head -12
done
