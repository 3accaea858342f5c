#!/bin/bash
# The GPU test suite alone (pytest -m gpu), log under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-gpu_tests}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; exit $rc
