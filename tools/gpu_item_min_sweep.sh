#!/bin/bash
# The 1/8 strip's automatic item size (RTMI_ITEM_MIN: the smallest item, in
# samples; the library default 24), twice each, interleaved: bench.py kernel ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-item_min}
mkdir -p $OUT
for rep in 1 2; do
  for im in ${ITEM_MINS:-16 20 24 32}; do
    RTMI_ITEM_MIN=$im timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 > $OUT/im${im}_$rep.json 2> $OUT/im${im}_$rep.err || { tail -3 $OUT/im${im}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/im${im}_$rep.json')); print('item_min $im strip8', d['roofline']['kernel_ms'], d['config']['tile'])"
  done
done
