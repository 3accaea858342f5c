#!/bin/bash
# NW quick check: parity tests, phase split (RTMI_NW_PHASES variant), both bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-nw_quick}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/nw_phases.py > $OUT/phases.txt 2>&1 || { tail -5 $OUT/phases.txt; exit 1; }
grep scene $OUT/phases.txt
for w in nw_motion_blur nw_final; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; a=json.load(open('$OUT/$w.json')); print('$w', a['ms_per_step'], a['value'], a['config'].get('accel'))"
done
