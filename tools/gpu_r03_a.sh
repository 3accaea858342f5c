#!/bin/bash
# Round 3, first pass: bit-exactness of the big-sphere variants, their A/B on
# config 2 and the 1/8 strip, and the config 4 / config 5 bench lines on HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03a}
mkdir -p $OUT
for v in $VARIANTS; do
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$v.so timeout -k 10 120 python -u tools/check_variant.py > $OUT/check_$v.txt 2>&1 || { tail -5 $OUT/check_$v.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/check_$v.txt)"
done
TAG=${TAG:-r03a}/ab LIBS="$LIBS" bash tools/gpu_ab_lib.sh || exit 1
for w in $WORKLOADS; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload $w > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['work_equivalent_frac'])"
done
