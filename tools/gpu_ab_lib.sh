#!/bin/bash
# A/B of library build variants (a_dive_into_ray_tracing_amd/lib/librtmi_<NAME>.so,
# made with `make -C a_dive_into_ray_tracing_amd/csrc variant NAME=.. VFLAGS=..`):
# LIBS="base eu6 ..." BENCH_ARGS="--accel grid" bash tools/gpu_ab_lib.sh
# Each variant: config 2 and the 1/8 strip, twice, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-ab_lib}
mkdir -p $OUT
for rep in 1 2; do
  for v in $LIBS; do
    lib=a_dive_into_ray_tracing_amd/lib/librtmi_$v.so; [ "$v" = base ] && lib=a_dive_into_ray_tracing_amd/lib/librtmi.so
    RTMI_LIBRARY=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only $BENCH_ARGS > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail -3 $OUT/${v}_$rep.err; exit 1; }
    RTMI_LIBRARY=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 $BENCH_ARGS > $OUT/${v}_s8_$rep.json 2> $OUT/${v}_s8_$rep.err || exit 1
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); s=json.load(open('$OUT/${v}_s8_$rep.json')); print('$v', d['roofline']['kernel_ms'], 'strip8', s['roofline']['kernel_ms'])"
  done
done
