#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== stats" && timeout -k 10 300 python tools/stats_run.py 2>&1 | grep -v amdgpu.ids
echo "== ab" && VARIANTS="librtmi.so librtmi_gp2.so librtmi_gp8.so librtmi_w8.so librtmi_gp2w8.so librtmi_pre.so" bash tools/ab_bench.sh
