#!/bin/bash
# Kernel-shape A/B on the 1/8 strip and the frame (grid accel): one wave per
# item (grid kernel), the persistent kernel (round 2; its block-job-pool leg
# was dropped with the pool in round 3)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-ab_kernel}; mkdir -p $OUT
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only $EXTRA > $OUT/$name.json 2> $OUT/$name.err || { tail -3 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  EXTRA="--strip-of 8" run s8_grid_$rep X=1
  EXTRA="--strip-of 8 --kernel persistent" run s8_pers_$rep X=1
  EXTRA="--kernel persistent" run f_pers_$rep X=1
done
