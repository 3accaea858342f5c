#!/bin/bash
# The queue kernel: its parity tests (tests/test_gpu_queue.py),
# then config 2 and the 1/8 strip through the grid kernel and the queue
# kernel, interleaved twice; QLIBS="<v> ..." adds library variants
# (lib/librtmi_<v>.so, e.g. other bin / pool sizes) run with --kernel queue.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-queue}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_queue.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_queue.log | tail -20; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, kernel, extra args; env LIB
  local name=$1 k=$2; shift 2
  RTMI_LIBRARY=${LIB:-} timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only \
    --kernel $k "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run grid_$rep grid || exit 1
  run queue_$rep queue || exit 1
  for v in $QLIBS; do LIB=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$v.so run ${v}_$rep queue || exit 1; done
  run grid_strip8_$rep grid --strip-of 8 || exit 1
  run queue_strip8_$rep queue --strip-of 8 || exit 1
done
