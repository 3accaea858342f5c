#!/bin/bash
# Round 3: the Next-Week GPU suite on the current tree, then an A/B of
# library variants on the Next-Week lines (LIBS, via gpu_ab_nw_lib.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_nwcheck}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_nw.log 2>&1
rc=$?; tail -3 $OUT/pytest_nw.log; [ $rc -eq 0 ] || exit $rc
[ -n "$LIBS" ] && { TAG=${TAG:-r03_nwcheck}/ab LIBS="$LIBS" bash tools/gpu_ab_nw_lib.sh || exit 1; }
exit 0
