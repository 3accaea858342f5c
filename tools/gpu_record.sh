#!/bin/bash
# The whole record of the current tree in one GPU call (B=<name>): smoke +
# GPU suite + bench line + 1/8 strip + rocprofv3 kernel trace (gpu_pass.sh),
# PMC passes (profile.sh), the write budget passes (gpu_writes.sh), configs 4
# and 5 (gpu_workloads.sh) and, with NW=1, the Next-Week lines
# (gpu_nw_lines.sh).  Outputs under gpurun_out/<B>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-record}
TAG=$B/pass bash tools/gpu_pass.sh || exit 1
TAG=$B/prof bash tools/profile.sh > gpurun_out/$B/profile.log 2>&1 || { tail -5 gpurun_out/$B/profile.log; exit 1; }
tail -3 gpurun_out/$B/profile.log
TAG=$B/writes bash tools/gpu_writes.sh > gpurun_out/$B/writes.log 2>&1 || { tail -5 gpurun_out/$B/writes.log; exit 1; }
tail -8 gpurun_out/$B/writes.log
TAG=$B/workloads bash tools/gpu_workloads.sh || exit 1
[ -n "$NW" ] && { TAG=$B/nw bash tools/gpu_nw_lines.sh || exit 1; }
exit 0
