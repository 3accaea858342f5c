#!/bin/bash
# A/B of Next-Week kernel variants (librtmi_<name>.so), both nw workloads, each in its own process.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nwab
for lib in ${VARIANTS:-librtmi.so}; do
  for wl in nw_motion_blur nw_final; do
    RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/$lib timeout -k 10 200 python bench.py --workload $wl --steps 2 --warmup 1 --nw-spp ${NWSPP:-256} > gpurun_out/nwab/${lib}_$wl.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/nwab/${lib}_$wl.json')); print('$lib', '$wl', d['value'], d['kernel_ms'], d['objects_bvh_nodes'])"
  done
done
