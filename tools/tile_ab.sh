#!/bin/bash
# Tile width A/B (automatic chunk) on config 2 and one rank's 1/8, 1/4, 1/2
# strips, each run twice to show the run-to-run spread.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-tab}
mkdir -p $OUT
run() {
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/s.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/s.json')); print(sys.argv[1:], d['roofline']['kernel_ms'])" "$@"
}
for rep in 1 2; do
  for tw in 8 16; do
    run --tile-w $tw
    for n in 8 4 2; do run --tile-w $tw --strip-of $n; done
  done
done
