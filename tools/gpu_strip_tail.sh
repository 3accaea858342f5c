#!/bin/bash
# 1/8 strip: long items first, a short-item tail (--chunk / --tail-spp / --tail-chunk), against the automatic schedule
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-strip_tail}; mkdir -p $OUT
for cfg in "0 -1 0" "42 84 7" "63 63 9" "32 100 10" "125 125 5" "48 52 4" "40 60 6"; do
  set -- $cfg
  n="c$1_t$2_k$3"
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 --chunk $1 --tail-spp $2 --tail-chunk $3 > $OUT/$n.json 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
