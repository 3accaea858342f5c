#!/bin/bash
# Bit-exactness of library variants (tests/test_gpu_parity.py with
# RTMI_LIBRARY = lib/librtmi_<v>.so, for every v of LIBS except base), then
# their interleaved A/B on config 2 and the 1/8 strip (tools/gpu_ab_lib.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-variants}
mkdir -p $OUT
for v in $LIBS; do
  [ "$v" = base ] && continue
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "variant $v: parity FAILED"; tail -20 $OUT/parity_$v.log; exit 1; }
  echo "variant $v: $(tail -1 $OUT/parity_$v.log)"
done
TAG=${TAG:-variants}/ab LIBS="$LIBS" bash tools/gpu_ab_lib.sh || exit 1
python tools/ab_summary.py $OUT/ab "$LIBS"
