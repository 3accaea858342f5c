#!/bin/bash
# GPU: the queue kernel's parity tests, then a config-2 A/B of grid vs queue
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-q}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_queue.log 2>&1
rc=$?; tail -15 $OUT/pytest_queue.log; [ $rc -eq 0 ] || exit $rc
for k in grid queue grid queue; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --kernel $k > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { tail $OUT/bench_$k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$k.json')); print('$k', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
