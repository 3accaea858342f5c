#!/bin/bash
# Per-wave timelines (RTMI_TRACE build, lib/librtmi_wavetrace.so — build it on
# the CPU first: python tools/variants.py build wavetrace) of the kernel shapes
# in KERNELS, whole frame and one rank's 1/8 strip.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
python tools/variants.py check wavetrace || exit 1
export TRACE_LIB=librtmi_wavetrace.so
OUT=gpurun_out/${TAG:-trace_ab}; mkdir -p $OUT
for k in ${KERNELS:-grid resident}; do
  for s in 1 8; do
    TRACE_ACCEL=grid timeout -k 10 180 python -u tools/trace_run.py $k $s > $OUT/trace_${k}_strip$s.txt 2>&1 || { tail $OUT/trace_${k}_strip$s.txt; exit 1; }
    head -7 $OUT/trace_${k}_strip$s.txt
  done
done
