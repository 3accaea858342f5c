#!/bin/bash
# Round 3: GPU tests on the current tree, then the ramp-down hand-off A/B
# (RTMI_HANDOFF / RTMI_HANDOFF_LANES; same library, same image) on the
# config-2 frame and one rank's 1/8 strip.
# LANES="16 24 40" TAG=.. SKIP_TESTS=1 bash tools/gpu_handoff_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-handoff_ab}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
B="python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only"
run() {  # name, extra bench args; env from the caller
  timeout -k 10 180 $B $2 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['roofline']['kernel_ms'], d['ms_per_step'])"
}
for rep in 1 2; do
  for shape in frame s8; do
    args=""; [ $shape = s8 ] && args="--strip-of 8"
    RTMI_HANDOFF=0 run ${shape}_off_$rep "$args"
    for l in ${LANES:-16 24 40}; do
      RTMI_HANDOFF=1 RTMI_HANDOFF_LANES=$l run ${shape}_l${l}_$rep "$args"
    done
  done
done
exit 0
