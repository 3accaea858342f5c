#!/bin/bash
# 1/8 strip (and the frame): automatic items plus a short-item tail phase of T samples, both phases
# block-flushed (round 3), against the automatic schedule without a tail.  TAILS="50 100 150"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-strip_tail2}; mkdir -p $OUT
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only"
for rep in 1 2; do
  for t in -1 ${TAILS:-50 100 150}; do
    timeout -k 10 120 $B --strip-of 8 --tail-spp $t > $OUT/s8_t${t}_$rep.json 2> $OUT/s8_t${t}_$rep.err || { tail -3 $OUT/s8_t${t}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/s8_t${t}_$rep.json')); print('strip8 tail $t', d['roofline']['kernel_ms'], d['config'].get('schedule'))"
  done
  for t in -1 ${FTAILS:-50}; do
    timeout -k 10 120 $B --tail-spp $t > $OUT/fr_t${t}_$rep.json 2> $OUT/fr_t${t}_$rep.err || { tail -3 $OUT/fr_t${t}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/fr_t${t}_$rep.json')); print('frame tail $t', d['roofline']['kernel_ms'])"
  done
done
