#!/bin/bash
# Generic InteractingLayer A/B (il_generic.hip build knobs): every tools/il_shape_bench.py shape
# forced onto the generic kernels, the in-tree library vs variant libraries under abv6/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RS_IL_FORCE_GENERIC=1
for v in base ${VARIANTS:-g_auto g_nt512 g_both}; do
  if [ $v = base ]; then L="RS_NONE=0"; else L="RS_LIB_PATH=abv6/$v.so"; fi
  env $L timeout -k 10 200 python tools/il_shape_bench.py 2048 > gpurun_out/gab_$v.log 2>&1 || { echo "fail $v"; exit 1; }
  echo "== $v"; grep "F=" gpurun_out/gab_$v.log
done
