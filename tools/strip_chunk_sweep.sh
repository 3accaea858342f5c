#!/bin/bash
# One rank's 1/8 strip of config 2 (BVH) over phase-1 chunk sizes whose item
# counts per tile are multiples of the block's 4 waves (block flush stays on).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sc
for tw in ${TILES:-8 16}; do
  for ch in ${CHUNKS:-7 14 16 18 21 25 32}; do
    timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --strip-of ${STRIP_OF:-8} --tile-w $tw --chunk $ch > gpurun_out/sc/s.json 2> gpurun_out/sc/s.err || { tail gpurun_out/sc/s.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sc/s.json')); print('tile_w', $tw, 'chunk', $ch, d['roofline']['kernel_ms'])"
  done
done
