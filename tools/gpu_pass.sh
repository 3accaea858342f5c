#!/bin/bash
# One GPU pass over the current tree: smoke, the GPU test suite (its
# statistical numbers land in gpurun_out/parity_stats.json), the default bench
# line, one rank's 1/8 strip, and a rocprofv3 kernel trace of the bench.
# Every GPU step has its own limit; the first failing step ends the script.
# TAG names the output directory; SKIP_TESTS=1 / SKIP_PROF=1 skip steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pass}
mkdir -p $OUT
rm -f gpurun_out/parity_stats.json
echo "== smoke" && timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/parity_stats.json $OUT/ 2>/dev/null
fi
echo "== bench" && timeout -k 10 400 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== strip 1/8" && timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exec-counts --strip-of 8 > $OUT/strip8.json 2> $OUT/strip8.err || exit 1
python -c "import json; d=json.load(open('$OUT/strip8.json')); print('strip8', d['ms_per_step'], d['roofline']['kernel_ms'], d['one_shot'])"
[ -n "$SKIP_PROF" ] && exit 0
echo "== rocprof kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only > $OUT/kt_bench.json 2> $OUT/kt.err || exit 1
cat $OUT/kt_bench.json
find $OUT/kt -name "*kernel_stats.csv" -exec head -6 {} \;
python3 tools/trace_busy.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) | tee $OUT/kt_busy.txt
