#!/bin/bash
# Persistent kernel (grid accel) on the 1/8 strip and the frame: item size sweep
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-pers_chunk}; mkdir -p $OUT
for c in 0 8 16 32 64; do
  timeout -k 10 120 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 --kernel persistent --chunk $c > $OUT/s8_$c.json 2> $OUT/s8_$c.err || { tail -3 $OUT/s8_$c.err; exit 1; }
  timeout -k 10 120 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only --kernel persistent --chunk $c > $OUT/f_$c.json 2> $OUT/f_$c.err || { tail -3 $OUT/f_$c.err; exit 1; }
  python -c "import json; a=json.load(open('$OUT/s8_$c.json')); b=json.load(open('$OUT/f_$c.json')); print('chunk $c', 'strip', a['roofline']['kernel_ms'], 'frame', b['roofline']['kernel_ms'])"
done
