#!/bin/bash
# Per-wave trace + phase clocks of the RTMI_TRACE build (lib/librtmi_trace.so,
# built on the CPU first: python tools/variants.py build trace): whole frame and
# the 1/8 strip.  A variant built from other sources is refused.
cd "$GRAFT_REPO_ROOT" || exit 1
python tools/variants.py check trace || exit 1
mkdir -p gpurun_out
TRACE_ACCEL=grid TRACE_PHASES=1 timeout -k 10 180 python -u tools/trace_run.py grid 1 > gpurun_out/trace_phases_frame.txt 2>&1 &&
TRACE_ACCEL=grid TRACE_PHASES=1 timeout -k 10 180 python -u tools/trace_run.py grid 8 > gpurun_out/trace_phases_strip8.txt 2>&1
rc=$?; head -9 gpurun_out/trace_phases_strip8.txt; exit $rc
