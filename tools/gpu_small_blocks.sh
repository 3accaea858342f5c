#!/bin/bash
# 2-wave grid-kernel blocks (lib/librtmi_w2.so) with the grid walked in global
# memory (RTMI_GRID_LDS_MAX=1: no LDS copy per block, so 16 blocks fit a CU):
# a finished wave frees its slots with one partner instead of three.  Against
# the product (4-wave blocks, grid in LDS) and the product with the global
# walk; config 2 frame and one rank's 1/8 strip, --pipeline 1 and 2, REPS times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
python tools/variants.py check w2 || exit 1
OUT=gpurun_out/${TAG:-small_blocks}; mkdir -p $OUT
W2=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_w2.so
run() {  # name, lib (- = product), lds max (- = default), bench args...
  local name=$1 lib=$2 lm=$3; shift 3
  local L=""; [ "$lib" != "-" ] && L=$W2
  local M=""; [ "$lm" != "-" ] && M=$lm
  RTMI_LIBRARY=$L RTMI_GRID_LDS_MAX=$M timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 3 \
    --no-cpu-baseline --no-exec-counts --timed-only "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
}
for rep in $(seq ${REPS:-2}); do
  for p in 1 2; do
    for so in 1 8; do
      sa=""; [ $so -gt 1 ] && sa="--strip-of $so"
      run lds4_p${p}_s${so}_$rep - - --pipeline $p $sa || exit 1
      run gmem4_p${p}_s${so}_$rep - 1 --pipeline $p $sa || exit 1
      run gmem2_p${p}_s${so}_$rep w2 1 --pipeline $p $sa || exit 1
    done
  done
done
