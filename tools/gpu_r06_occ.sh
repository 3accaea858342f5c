#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_occ; mkdir -p $OUT
run() {
  local name=$1 lib=$2; shift 2
  local L=""; [ "$lib" != "-" ] && L=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$lib.so
  local args=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
  env RTMI_LIBRARY=$L "${args[@]}" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts \
    --timed-only --pipeline 1 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run grid_$rep - X=1 -- --kernel grid || exit 1
  run rw8_1024_$rep rw8 X=1 -- --kernel resident || exit 1
  run rw8_960_$rep rw8 RTMI_RES_BLOCKS=960 -- --kernel resident || exit 1
  run rw8_896_$rep rw8 RTMI_RES_BLOCKS=896 -- --kernel resident || exit 1
  run rw4_$rep rw4 X=1 -- --kernel resident || exit 1
  run rw4_s8_$rep rw4 X=1 -- --kernel resident --strip-of 8 || exit 1
done
