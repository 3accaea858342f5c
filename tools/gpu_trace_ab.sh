#!/bin/bash
# Per-wave timelines (RTMI_TRACE build, lib/librtmi_trace.so — build it first:
# make -C a_dive_into_ray_tracing_amd/csrc variant NAME=trace VFLAGS=-DRTMI_TRACE=1)
# of the kernel shapes in KERNELS, whole frame and one rank's 1/8 strip.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-trace_ab}; mkdir -p $OUT
for k in ${KERNELS:-grid resident}; do
  for s in 1 8; do
    TRACE_ACCEL=grid timeout -k 10 180 python -u tools/trace_run.py $k $s > $OUT/trace_${k}_strip$s.txt 2>&1 || { tail $OUT/trace_${k}_strip$s.txt; exit 1; }
    head -7 $OUT/trace_${k}_strip$s.txt
  done
done
