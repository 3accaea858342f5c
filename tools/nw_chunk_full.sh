#!/bin/bash
# Next-Week item size A/B (RTMI_NW_CHUNK) at the bench's full spp; ms per render.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nwc
for w in nw_motion_blur nw_final; do
  for ch in ${CHUNKS:-32 8 12 16 24}; do
    RTMI_NW_CHUNK=$ch timeout -k 10 200 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nwc/f.json 2> gpurun_out/nwc/f.err || { tail gpurun_out/nwc/f.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nwc/f.json')); print('$w', 'chunk', $ch, d['ms_per_step'], d['value'])"
  done
done
