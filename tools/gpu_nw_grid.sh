#!/bin/bash
# Next-Week grid: GPU parity (all NW tests) then the two NW bench lines with
# the automatic structure and with the BVH forced
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-nw_grid}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for w in nw_motion_blur nw_final; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  timeout -k 10 300 python -u bench.py --workload $w --nw-accel bvh --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/${w}_bvh.json 2> $OUT/${w}_bvh.err || { tail -5 $OUT/${w}_bvh.err; exit 1; }
  python -c "import json; a=json.load(open('$OUT/$w.json')); b=json.load(open('$OUT/${w}_bvh.json')); print('$w', a['ms_per_step'], a['value'], a['config'].get('accel'), '| bvh', b['ms_per_step'], b['value'])"
done
