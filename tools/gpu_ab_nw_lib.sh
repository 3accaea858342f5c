#!/bin/bash
# A/B of library variants on the Next-Week lines (motion blur 500 spp, final 256 spp), interleaved, twice
# LIBS="base nwold" bash tools/gpu_ab_nw_lib.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-ab_nw_lib}; mkdir -p $OUT
for rep in 1 2; do
  for v in $LIBS; do
    lib=a_dive_into_ray_tracing_amd/lib/librtmi_$v.so; [ "$v" = base ] && lib=a_dive_into_ray_tracing_amd/lib/librtmi.so
    RTMI_LIBRARY=$PWD/$lib timeout -k 10 200 python -u bench.py --workload nw_motion_blur --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${v}_mb_$rep.json 2> $OUT/${v}_mb_$rep.err || { tail -3 $OUT/${v}_mb_$rep.err; exit 1; }
    RTMI_LIBRARY=$PWD/$lib timeout -k 10 200 python -u bench.py --workload nw_final --nw-spp 256 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${v}_fs_$rep.json 2> $OUT/${v}_fs_$rep.err || { tail -3 $OUT/${v}_fs_$rep.err; exit 1; }
    python -c "import json; a=json.load(open('$OUT/${v}_mb_$rep.json')); b=json.load(open('$OUT/${v}_fs_$rep.json')); print('$v', 'mb', a['kernel_ms'], 'final256', b['kernel_ms'])"
  done
done
