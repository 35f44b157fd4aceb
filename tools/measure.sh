#!/bin/bash
# One parameterised GPU-box runner for the round's measurements (replaces the single-use run
# scripts of earlier rounds).  Each step runs under its own time limit; the first failing step
# ends the run (no GPU step after a fault, a timeout or an abort).
#
#   bash tools/measure.sh OUTDIR step [step ...]
#     gputest      pytest -m gpu (whole suite, one process)
#     bench        default bench line (200 steps, CPU baseline, config-1 leg)
#     driver       the driver's command: --steps 20 --warmup 5
#     trace        rocprofv3 --kernel-trace --stats of bench.py --steps 50
#     pmc          FETCH_SIZE / WRITE_SIZE passes over bench.py -> OUTDIR/il_bwd_traffic.json
#     workloads    configs 3-5 bench lines (bench.py --workload multi_head | din | staytime)
#     wltrace      rocprofv3 kernel traces of the configs 3-5 timed steps (tools/prof_steps.py)
#     small        per-GPU batch 512 .. 4096 (tools/small_batch.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=$1; shift
mkdir -p "$D"
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "ABORT rc=$rc: $*"; exit $rc; fi; }
line() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); r=d.get('roofline') or {}; print('$2', d['value'], d['ms_per_step'], r.get('frac'), r.get('launch_us'))"; }
for s in "$@"; do
  case $s in
    gputest)
      step 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$D/pytest_gpu.log" 2>&1
      tail -3 "$D/pytest_gpu.log" ;;
    bench)
      step 400 python3 bench.py > "$D/bench_default.log" 2>&1
      line "$D/bench_default.log" bench ;;
    driver)
      step 200 python3 bench.py --steps 20 --warmup 5 > "$D/bench_20_5.log" 2>&1
      line "$D/bench_20_5.log" driver ;;
    trace)
      step 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --kernel-reps 50 > "$D/bench_traced.log" 2>&1
      line "$D/bench_traced.log" traced ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        step 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$D/pmc_$c" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --kernel-reps 5 > "$D/pmc_$c.log" 2>&1
      done
      step 60 python3 tools/il_traffic.py "$D" 4096 "$D/il_bwd_traffic.json" | cut -c1-300 ;;
    workloads)
      for w in multi_head din staytime; do
        step 400 python3 bench.py --workload $w --steps 50 --warmup 10 > "$D/wl_$w.log" 2>&1
        line "$D/wl_$w.log" $w
      done ;;
    wltrace)
      for w in multi_head din staytime; do
        step 400 rocprofv3 --kernel-trace --output-format csv -d "$D/wlt_$w" -o run -- python3 bench.py --workload $w --steps 30 --warmup 10 --trace-markers --no-cpu-baseline --kernel-reps 5 > "$D/wlt_$w.log" 2>&1
        step 60 python3 tools/prof_steps.py "$D/wlt_$w" 30 0 "$D/steps_$w.json" | head -25
      done ;;
    small)
      OUT="$D/small_batch" step 1000 bash tools/small_batch.sh ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
