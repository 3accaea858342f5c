#!/bin/bash
# Kernel shape A/B with the BVH: grid (auto) vs the persistent continuous job
# stream, on config 2 and one rank's 1/8 strip, over chunk sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-pab}
mkdir -p $OUT
run() {
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/s.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/s.json')); print(sys.argv[1:], d['roofline']['kernel_ms'])" "$@"
}
run --chunk 125
run --strip-of 8 --tile-w 16 --chunk 25
run --kernel persistent
run --strip-of 8 --kernel persistent
for ch in 4 8 16 32; do
  run --strip-of 8 --kernel persistent --chunk $ch
  run --kernel persistent --chunk $ch
done
