#!/bin/bash
# Round-6 PMC evidence, each counter group in its own kernel-trace-only pass:
#   step traffic of the config-2 step (FETCH_SIZE / WRITE_SIZE over bench.py: every launch of the
#   step) -> il_bwd_traffic.json (the roofline launch) + step_traffic.json (all four launches);
#   SQ counters of the config-2 IL backward (tools/pmc_il_sq.sh) and of the config-3 many-field
#   IL backward (tools/pmc_il_large.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${D:-gpurun_out/r06_ev}; mkdir -p $D; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $D/pmc_$c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16 --kernel-reps 5 > $D/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $D/pmc_$c.log; exit 1; }
  ln -sfn pmc_$c $D/step_dz_$c
done
timeout -k 10 60 python3 tools/il_traffic.py $D 4096 $D/il_bwd_traffic.json | cut -c1-200 || exit 1
timeout -k 10 60 python3 tools/step_traffic.py $D $D/step_traffic.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$D/step_traffic.json'))['dz']; print({k: (v['hbm_mb'] if isinstance(v, dict) else v) for k, v in d.items()})"
PMC_DIR=$D/sq4 timeout -k 10 300 bash tools/pmc_il_sq.sh > $D/sq4.txt 2>&1 || { tail -5 $D/sq4.txt; exit 1; }
tail -12 $D/sq4.txt
timeout -k 10 300 bash tools/pmc_il_large.sh > $D/sq_large.txt 2>&1 || { tail -5 $D/sq_large.txt; exit 1; }
cp -r gpurun_out/pmc_ill $D/ 2>/dev/null
tail -20 $D/sq_large.txt
