#!/bin/bash
# A/B of the closest-hit structures on config 2 and the 1/8 strip: BVH vs
# uniform grid (same image), plus grid densities (RTMI_GRID_CELLS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-ab_accel}
mkdir -p $OUT
for acc in bvh grid; do
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --accel $acc > $OUT/$acc.json 2> $OUT/$acc.err || { tail $OUT/$acc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$acc.json')); r=d['roofline']; print('$acc', d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('counts'))"
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --accel $acc --strip-of 8 > $OUT/${acc}_s8.json 2> $OUT/${acc}_s8.err || exit 1
  python -c "import json; d=json.load(open('$OUT/${acc}_s8.json')); print('$acc strip8', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
for c in 0.5 2 4; do
  RTMI_GRID_CELLS=$c timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --accel grid > $OUT/grid_c$c.json 2> $OUT/grid_c$c.err || exit 1
  python -c "import json; d=json.load(open('$OUT/grid_c$c.json')); print('grid cells/sphere $c', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
