#!/bin/bash
# One rank's 1/8 strip (and the whole frame) under two-phase schedules:
# TAILS = "tail_spp:tail_chunk" pairs (0:0 = one phase).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tc in ${TAILS:-0:0 100:10 60:6 150:15}; do
  t=${tc%%:*}; c=${tc##*:}
  for args in "--strip-of 8" ""; do
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tail-spp $t --tail-chunk $c $args > gpurun_out/tail.json 2> gpurun_out/tail.err || { tail gpurun_out/tail.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tail.json')); print('tail', '$tc', '$args', d['roofline']['kernel_ms'])"
  done
done
