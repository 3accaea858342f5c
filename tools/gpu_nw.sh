#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/nw
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/nw/pytest_nw.log 2>&1
rc=$?; tail -25 gpurun_out/nw/pytest_nw.log; exit $rc
