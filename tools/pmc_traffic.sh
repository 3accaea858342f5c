#!/bin/bash
# HBM-side traffic of the render kernels on config 2: FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes (no tracing), then per-dispatch means.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-traffic}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only $BENCH_ARGS"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > $OUT/pmc1.json 2> $OUT/pmc1.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > $OUT/pmc2.json 2> $OUT/pmc2.err || exit $?
python3 tools/pmc_summary.py $OUT | tee $OUT/summary.txt
