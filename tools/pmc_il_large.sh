#!/bin/bash
# SQ counters of the config-3 many-field IL kernels (tools/il_large_bench.py), one pass per set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_ill
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_ill/p$i -o run -- \
    python3 tools/il_large_bench.py > gpurun_out/pmc_ill/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_ill/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_ill/p*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'bwd_kernel' in r['Kernel_Name']:
            acc[(r['Dispatch_Id'], r['Counter_Name'])].append(float(r['Counter_Value']))
    per = collections.defaultdict(list)
    for (d, c), v in acc.items():
        per[c].append(sum(v))
    for c, v in sorted(per.items()):
        print(f"{c:24s} n={len(v):3d} last={v[-1]:.4g} first={v[0]:.4g}")
PY
