#!/bin/bash
# Round 3: RTIOW parity + Next-Week GPU suites on the current tree, then an
# A/B of library variants (LIBS) on config 2 and the 1/8 strip
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_suite}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nw_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
[ -n "$LIBS" ] && { TAG=${TAG:-r03_suite}/ab LIBS="$LIBS" bash tools/gpu_ab_lib.sh || exit 1; }
exit 0
