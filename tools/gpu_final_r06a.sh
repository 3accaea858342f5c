#!/bin/bash
# Round 6 final record, part A (B=<name>, default r06_final): smoke + GPU suite +
# bench line + 1/8 strip + rocprofv3 kernel trace (gpu_pass.sh), the PMC passes
# (profile.sh) and the write budget passes (gpu_writes.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-r06_final}
mkdir -p gpurun_out/$B
TAG=$B/pass bash tools/gpu_pass.sh || exit 1
TAG=$B/prof bash tools/profile.sh > gpurun_out/$B/profile.log 2>&1 || { tail -5 gpurun_out/$B/profile.log; exit 1; }
tail -3 gpurun_out/$B/profile.log
TAG=$B/writes bash tools/gpu_writes.sh > gpurun_out/$B/writes.log 2>&1 || { tail -5 gpurun_out/$B/writes.log; exit 1; }
tail -8 gpurun_out/$B/writes.log
