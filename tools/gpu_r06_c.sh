#!/bin/bash
# round 6: the Next-Week signed-zero walk test and the resident kernel's
# tests, then the tile-locality A/B of the grid kernel (chunk-major items)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06_c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -k signed_zero tests/test_gpu_resident.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -30; [ $rc -eq 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
run() {  # name, lib, env..., then bench args after --
  local name=$1 lib=$2; shift 2
  local L=""; [ "$lib" != "-" ] && L=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$lib.so
  env RTMI_LIBRARY=$L "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts \
    --timed-only --pipeline 1 > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run grid_$rep - X=1 || exit 1
  run grid_noflush_$rep - RTMI_BLOCK_FLUSH=0 || exit 1
  run cmaj_$rep cmaj X=1 || exit 1
done
