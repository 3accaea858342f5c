#!/bin/bash
# A/B of kernel shapes and library variants on config 2 and one rank's 1/8
# strip, single launches (--pipeline 1).  AB="name:kernel:lib ..." (lib: a
# lib/librtmi_<lib>.so variant or "-" for librtmi.so); REPS repetitions,
# interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_kernels}
mkdir -p $OUT
run() {  # name, kernel, lib, extra args
  local name=$1 k=$2 lib=$3; shift 3
  local L=""; [ "$lib" != "-" ] && L=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$lib.so
  RTMI_LIBRARY=$L timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts \
    --timed-only --pipeline 1 --kernel $k "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in $(seq ${REPS:-2}); do
  for spec in $AB; do
    IFS=: read n k l <<< "$spec"
    run ${n}_frame_$rep $k $l || exit 1
    run ${n}_strip8_$rep $k $l --strip-of 8 || exit 1
  done
done
