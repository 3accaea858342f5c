#!/bin/bash
# Quick GPU pass for a kernel change: smoke, a pytest selection (PYTEST_K,
# default the RTIOW parity file), the config-2 bench (no CPU baseline) and one
# rank's 1/8 strip.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
echo "== smoke" && timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo "== pytest ${PYTEST_SEL:-tests/test_gpu_parity.py}"
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_parity.py} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest.log | head -20; exit $rc; }
echo "== bench" && timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'bf', d['roofline']['brute_force']['kernel_ms'])"
echo "== strip 1/8" && timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --strip-of 8 $BENCH_ARGS > $OUT/strip8.json 2> $OUT/strip8.err || exit 1
python -c "import json; d=json.load(open('$OUT/strip8.json')); print('strip8', d['ms_per_step'], d['roofline']['kernel_ms'])"
