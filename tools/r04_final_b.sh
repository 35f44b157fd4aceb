#!/bin/bash
# round-4 final measurements: default / driver-length / long bench lines, rocprofv3 kernel trace +
# stats of the default command, PMC traffic of the IL backward (il_bench) and of every step
# kernel in both dW1 modes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final
mkdir -p $D
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; }
step 300 python3 bench.py > $D/bench_default.log 2>&1
grep '^{' $D/bench_default.log | cut -c1-300
step 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_20_5.log 2>&1
grep '^{' $D/bench_20_5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('20/5', d['ms_per_step'], d['value'], d['roofline']['frac'])"
step 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --kernel-reps 50 > $D/bench_traced.log 2>&1
echo traced ok
for c in FETCH_SIZE WRITE_SIZE; do
  IL_BENCH_ONLY=push_hot_base_saved REPS=10 step 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/pmc_$c -o run -- python3 tools/il_bench.py > $D/pmc_$c.log 2>&1
  step 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/step_dz_$c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --kernel-reps 2 > $D/step_dz_$c.log 2>&1
  RS_HEAD_W1_PARTIALS=1 step 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/step_part_$c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --kernel-reps 2 > $D/step_part_$c.log 2>&1
  echo pmc $c ok
done
python3 tools/step_traffic.py $D $D/step_traffic.json | tail -30
python3 tools/traffic_json.py $D $D/il_bwd_traffic.json | cut -c1-300
BATCHES="2048" OUT=$D/small_batch_2048 bash tools/small_batch.sh
