#!/bin/bash
# The resident grid kernel: its parity tests
# (tests/test_gpu_resident.py), then config 2 and one rank's 1/8 strip through
# the grid kernel and the resident kernel, single launches (--pipeline 1) and
# overlapping steps (--pipeline 2), interleaved REPS times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-resident}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_resident.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_resident.log | tail -30; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, kernel, extra args
  local name=$1 k=$2; shift 2
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only \
    --kernel $k "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['launch_ms_mean'])"
}
for rep in $(seq ${REPS:-2}); do
  for k in grid resident; do
    run ${k}_p1_$rep $k --pipeline 1 || exit 1
    run ${k}_strip8_p1_$rep $k --pipeline 1 --strip-of 8 || exit 1
    run ${k}_p2_$rep $k || exit 1
    run ${k}_strip8_p2_$rep $k --strip-of 8 || exit 1
  done
done
