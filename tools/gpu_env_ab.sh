#!/bin/bash
# A/B of environment settings on config 2 and the 1/8 strip (ENVSETS="A=1|A=2|..."),
# twice each, interleaved: kernel ms (HIP events, mean of 10 timed launches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-env_ab}
mkdir -p $OUT
IFS='|' read -r -a SETS <<< "$ENVSETS"
for rep in 1 2; do
  for i in "${!SETS[@]}"; do
    env ${SETS[$i]} timeout -k 10 150 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only > $OUT/set${i}_$rep.json 2> $OUT/set${i}_$rep.err || { tail -3 $OUT/set${i}_$rep.err; exit 1; }
    env ${SETS[$i]} timeout -k 10 150 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 > $OUT/set${i}_s8_$rep.json 2> $OUT/set${i}_s8_$rep.err || exit 1
    python -c "import json; d=json.load(open('$OUT/set${i}_$rep.json')); s=json.load(open('$OUT/set${i}_s8_$rep.json')); print('[${SETS[$i]}]', d['roofline']['kernel_ms'], 'strip8', s['roofline']['kernel_ms'])"
  done
done
