#!/bin/bash
# Grid density sweep (RTMI_GRID_CELLS = cells per small sphere) on config 2
# and the 1/8 strip, grid accel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-grid_sweep}
mkdir -p $OUT
for c in 0.2 0.3 0.5 0.7 1.0; do
  RTMI_GRID_CELLS=$c timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --accel grid > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  RTMI_GRID_CELLS=$c timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --accel grid --strip-of 8 > $OUT/s8_c$c.json 2> $OUT/s8_c$c.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c$c.json')); s=json.load(open('$OUT/s8_c$c.json')); print('cells/sphere $c', d['roofline']['kernel_ms'], 'strip8', s['roofline']['kernel_ms'])"
done
