#!/bin/bash
# NW grid density sweep on the motion-blur scene (RTMI_NW_GRID_CELLS = cells per object), BVH beside it
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-nw_grid_sweep}; mkdir -p $OUT
for c in bvh 0.25 0.5 1 2 4; do
  if [ $c = bvh ]; then A="--nw-accel bvh"; E=""; else A="--nw-accel grid"; E="RTMI_NW_GRID_CELLS=$c"; fi
  env $E timeout -k 10 300 python -u bench.py --workload nw_motion_blur --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts $A > $OUT/mb_$c.json 2> $OUT/mb_$c.err || { tail -5 $OUT/mb_$c.err; exit 1; }
  python -c "import json; a=json.load(open('$OUT/mb_$c.json')); print('$c', a['ms_per_step'], a['config'].get('accel'), a['config'].get('grid_dims'), a['config'].get('grid_max_cell'))"
done
