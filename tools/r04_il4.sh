#!/bin/bash
# round-4 bwd4 evidence: per-phase stamp shares (stamps build) + SQ counters for the config-2
# push variant (the step's kernel), B = 4096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STAMPS_LIB=_gpuvar/librecsys_stamps.so ONLY=push_hot_base_saved OUT=gpurun_out/r04_il4 bash tools/prof_il.sh
