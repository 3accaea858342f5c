#!/bin/bash
# Walk counters of the RTMI_STATS build (tools/bvh_stats.py grid) and
# the phase clocks of the RTMI_TRACE build (tools/gpu_trace_phases.sh) on the
# current tree: OUT=gpurun_out/<tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-phases}
mkdir -p $OUT
timeout -k 10 120 python -u tools/bvh_stats.py grid > $OUT/grid_stats.txt 2>&1 || { tail -5 $OUT/grid_stats.txt; exit 1; }
cat $OUT/grid_stats.txt
bash tools/gpu_trace_phases.sh || exit 1
mv gpurun_out/trace_phases_frame.txt gpurun_out/trace_phases_strip8.txt $OUT/
head -5 $OUT/trace_phases_frame.txt
