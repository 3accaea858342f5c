#!/bin/bash
# Round 3: GPU test suite on the current tree, bit-exactness of library
# variants, their A/B (config 2 + 1/8 strip) and optional workload lines.
# VARIANTS="eu7 big8" LIBS="old base eu7" WORKLOADS="config4 config5" TAG=.. bash tools/gpu_r03_b.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03b}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/parity_stats.json $OUT/ 2>/dev/null
fi
for v in $VARIANTS; do
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$v.so timeout -k 10 120 python -u tools/check_variant.py > $OUT/check_$v.txt 2>&1 || { tail -5 $OUT/check_$v.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/check_$v.txt)"
done
[ -n "$LIBS" ] && { TAG=${TAG:-r03b}/ab LIBS="$LIBS" bash tools/gpu_ab_lib.sh || exit 1; }
for w in $WORKLOADS; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload $w > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['work_equivalent_frac'])"
done
exit 0
