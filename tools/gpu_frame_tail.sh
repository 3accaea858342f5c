#!/bin/bash
# Config-2 frame: automatic schedule vs a short-item tail phase (--tail-spp / --tail-chunk)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-frame_tail}; mkdir -p $OUT
for rep in 1 2; do
for cfg in "0 -1 0" "0 25 5" "0 50 10" "0 100 25" "0 40 4"; do
  set -- $cfg
  n="c$1_t$2_k$3_$rep"
  timeout -k 10 120 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --chunk $1 --tail-spp $2 --tail-chunk $3 > $OUT/$n.json 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
done
