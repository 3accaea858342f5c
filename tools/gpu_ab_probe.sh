#!/bin/bash
# A/B of the cost probe: steady state with the previous render's map (mode 1),
# probing before every render (mode 2), never probing (mode 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/ab_probe
mkdir -p $OUT
for m in 1 2 0 1 2; do
  RTMI_ORDER_PROBE=$m timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts > $OUT/m$m.json 2> $OUT/m$m.err || exit 1
  python -c "import json; d=json.load(open('$OUT/m$m.json')); print('mode $m', d['ms_per_step'], d['roofline']['kernel_ms'], d['one_shot'])"
done
RTMI_ORDER_PROBE=1 timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --strip-of 8 > $OUT/s8.json 2>&1 || exit 1
python -c "import json; d=json.load(open('$OUT/s8.json')); print('strip8', d['ms_per_step'], d['roofline']['kernel_ms'], d['one_shot'])"
