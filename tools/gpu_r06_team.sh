#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_team; mkdir -p $OUT
RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_rteam.so timeout -k 10 120 python -u -c "
import numpy as np, a_dive_into_ray_tracing_amd as rt
w=rt.random_scene(); cam=rt.final_camera(1.5)
a=rt.Renderer(w,0); a.set_kernel('grid'); ia=a.render(cam,1200,800,64,50,1984); a.close()
b=rt.Renderer(w,0); b.set_kernel('resident'); ib=b.render(cam,1200,800,64,50,1984); s=b.last_schedule(); b.close()
print('team image == grid image:', np.array_equal(ia,ib), s)
assert np.array_equal(ia,ib)
" || exit 1
run() {
  local name=$1 lib=$2; shift 2
  local L=""; [ "$lib" != "-" ] && L=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$lib.so
  RTMI_LIBRARY=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts \
    --timed-only --pipeline 1 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run grid_$rep - --kernel grid || exit 1
  run team_$rep rteam --kernel resident || exit 1
  run grid_s8_$rep - --kernel grid --strip-of 8 || exit 1
  run team_s8_$rep rteam --kernel resident --strip-of 8 || exit 1
done
