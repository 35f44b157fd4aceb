#!/bin/bash
# round-4 final: the whole GPU test suite (one process, per-test timeouts) and smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/r04_final
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; tail -3 $D/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $D/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
rc=$?; tail -2 $D/smoke.log; exit $rc
