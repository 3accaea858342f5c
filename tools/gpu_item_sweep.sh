#!/bin/bash
# Item-size sweep of the grid kernel's automatic schedule (RTMI_ITEM_MIN /
# RTMI_WANT_ITEMS; same image): one rank's 1/8 strip and the config-2 frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-item_sweep}
mkdir -p $OUT
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only"
for m in ${MINS:-12 16 24 32}; do
  RTMI_ITEM_MIN=$m timeout -k 10 120 $B --strip-of 8 > $OUT/s8_min$m.json 2> $OUT/s8_min$m.err || exit 1
  python -c "import json; d=json.load(open('$OUT/s8_min$m.json')); print('strip8 item_min $m', d['roofline']['kernel_ms'])"
done
for w in ${WANTS:-30000 60000 120000}; do
  RTMI_WANT_ITEMS=$w timeout -k 10 120 $B > $OUT/fr_want$w.json 2> $OUT/fr_want$w.err || exit 1
  python -c "import json; d=json.load(open('$OUT/fr_want$w.json')); print('frame want_items $w', d['roofline']['kernel_ms'])"
done
