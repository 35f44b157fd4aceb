#!/bin/bash
# per-phase stamps of the IL kernels (wide / wave variants), diagnostic build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RS_LIB_PATH=recommendsystem_amd/librecsys_amd_stamps.so timeout -k 10 200 python3 tools/il_wide_stamps.py > gpurun_out/il_stamps.txt 2>&1
rc=$?; cat gpurun_out/il_stamps.txt; exit $rc
