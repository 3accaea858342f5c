#!/bin/bash
# Tile shapes (TILES = tile widths) on the whole frame and one rank's 1/8 strip.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tw in ${TILES:-8 16 32 64}; do
  for args in "--strip-of 8" ""; do
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tile-w $tw $args > gpurun_out/tile.json 2> gpurun_out/tile.err || { tail gpurun_out/tile.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tile.json')); print('tile_w', $tw, '$args', d['roofline']['kernel_ms'])"
  done
done
