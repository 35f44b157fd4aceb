#!/bin/bash
# multi-hot push tile size (RS_MH_THREADS builds in abv6/): parity test per variant, then the
# config-3 push kernel alone under rocprofv3 (tools/push_prof.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in abv6/*.so; do
  RS_LIB_PATH=$so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "multi_hot_push or sparse_push" -x -q --timeout 120 --timeout-method thread > gpurun_out/mh_$(basename $so .so).log 2>&1 || { echo "$so parity failed"; tail -20 gpurun_out/mh_$(basename $so .so).log; exit 1; }
  echo "$so parity: $(tail -1 gpurun_out/mh_$(basename $so .so).log)"
done
S="RS_NONE=0"; for so in abv6/*.so; do S="$S RS_LIB_PATH=$so"; done
SETTINGS="$S" CASES="c3 c3_scan" OUT=gpurun_out/mh_prof bash tools/push_prof.sh
