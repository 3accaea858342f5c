#!/bin/bash
# Item-size A/B on the 1/8 strip and the frame (grid accel): RTMI_WANT_ITEMS x RTMI_ITEM_MIN
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-strip_items}
mkdir -p $OUT
IFS=,; for cfg in ${CFGS:-60000 24,120000 12}; do IFS=" "
  set -- $cfg
  RTMI_WANT_ITEMS=$1 RTMI_ITEM_MIN=$2 timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 > $OUT/s8_$1_$2.json 2> $OUT/s8_$1_$2.err || exit 1
  RTMI_WANT_ITEMS=$1 RTMI_ITEM_MIN=$2 timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only > $OUT/f_$1_$2.json 2> $OUT/f_$1_$2.err || exit 1
  python -c "import json; s=json.load(open('$OUT/s8_$1_$2.json')); f=json.load(open('$OUT/f_$1_$2.json')); print('want $1 min $2: strip8', s['roofline']['kernel_ms'], 'frame', f['roofline']['kernel_ms'])"
done
