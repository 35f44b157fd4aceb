#!/bin/bash
# Round-6 same-box A/B of kernel variants (built here into abv6/ with RS_LIB_OUT + -D flags):
#   bash tools/r06_ab.sh OUTDIR TESTS "label:ENV=... " ...
# TESTS: a pytest -k/-path spec ("-" = none) run first on the in-tree library; then the stamps of
# abv6/st_*.so (if any) and REPS interleaved bench runs per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=$1; shift; T=$1; shift
mkdir -p "$D"
export TMPDIR=/tmp
if [ "$T" != "-" ]; then
  timeout -k 10 900 python3 -u -m pytest $T -x -q --timeout 200 --timeout-method thread > "$D/pytest.log" 2>&1
  rc=$?; tail -3 "$D/pytest.log"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" "$D/pytest.log" | head -20; exit $rc; }
fi
for so in abv6/st_*.so; do
  [ -e "$so" ] || continue
  n=$(basename "$so" .so)
  RS_LIB_PATH=$so timeout -k 10 120 python3 tools/il_stamps.py > "$D/stamps_$n.txt" 2>&1 || { echo "stamps $n failed"; tail -5 "$D/stamps_$n.txt"; exit 1; }
  echo "== $n"; grep -v amdgpu.ids "$D/stamps_$n.txt"
done
[ $# -gt 0 ] && REPS=${REPS:-3} STEPS=${STEPS:-300} timeout -k 10 900 bash tools/ab_bench.sh "$@" | tee "$D/ab.txt"
exit ${PIPESTATUS[0]}
