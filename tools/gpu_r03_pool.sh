#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r03c_pool
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_parity.log 2>&1
rc=$?; tail -3 $OUT/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
TAG=r03c_pool/ab LIBS="head base pool7" bash tools/gpu_ab_lib.sh
