#!/bin/bash
# Round 3: exhaustive exact-math test + the RTIOW parity suite on the current
# tree, then an A/B of library variants (LIBS, via gpu_ab_lib.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_math}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_parity.log 2>&1
rc=$?; tail -3 $OUT/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
[ -n "$LIBS" ] && { TAG=${TAG:-r03_math}/ab LIBS="$LIBS" bash tools/gpu_ab_lib.sh || exit 1; }
exit 0
