#!/bin/bash
# Round 4: the record-slot grid layout — GPU suite on the current library,
# then the interleaved A/B against the previous one (LIBS="r4b base").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_slots}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
TAG=${TAG:-r04_slots}/ab LIBS="${LIBS:-r4b base}" bash tools/gpu_ab_lib.sh || exit 1
python tools/ab_summary.py $OUT/ab "${LIBS:-r4b base}"
