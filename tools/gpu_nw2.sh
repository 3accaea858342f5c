#!/bin/bash
# Next-Week GPU pass: parity tests (incl. the CLI), the two nw bench lines, a
# rocprofv3 kernel trace of the final-scene bench; then the RTIOW 1/8-strip
# chunk sweep (scaling analysis).  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-nw2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_nw.log 2>&1
rc=$?; grep -E "passed|failed|nw final" $OUT/pytest_nw.log | tail -3; [ $rc -eq 0 ] || exit $rc
echo "== nw bench"
timeout -k 10 300 python -u bench.py --workload nw_motion_blur --steps 3 --warmup 1 > $OUT/nw_mb.json 2> $OUT/nw_mb.err || exit 1
cat $OUT/nw_mb.json
timeout -k 10 300 python -u bench.py --workload nw_final --steps 3 --warmup 1 > $OUT/nw_final.json 2> $OUT/nw_final.err || exit 1
cat $OUT/nw_final.json
echo "== rocprof nw_final"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --workload nw_final --steps 2 --warmup 1 > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
find $OUT/kt -name "*kernel_stats.csv" -exec head -4 {} \;
if [ -n "$SWEEP" ]; then
  echo "== strip 1/8 chunk sweep"
  for c in 8 12 16 24 32; do
    timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --strip-of 8 --chunk $c > $OUT/strip8_c$c.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$OUT/strip8_c$c.json')); print('chunk', $c, d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
fi
