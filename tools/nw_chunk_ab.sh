#!/bin/bash
# Next-Week item size A/B (RTMI_NW_CHUNK) on the motion-blur and final scenes at 256 spp; kernel ms.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nwc
for w in nw_motion_blur nw_final; do
  for ch in ${CHUNKS:-32 8 16 64 128}; do
    RTMI_NW_CHUNK=$ch timeout -k 10 200 python bench.py --workload $w --nw-spp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/nwc/s.json 2> gpurun_out/nwc/s.err || { tail gpurun_out/nwc/s.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nwc/s.json')); print('$w', 'chunk', $ch, d['ms_per_step'], d['value'])"
  done
done
