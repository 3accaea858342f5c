#!/bin/bash
# Next-Week lines (executed-work roofline) on the current tree and,
# for comparison, with an older library (NWLIBS="base old").
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-nw_lines}
mkdir -p $OUT
for v in ${NWLIBS:-base}; do
  lib=a_dive_into_ray_tracing_amd/lib/librtmi_$v.so; [ "$v" = base ] && lib=a_dive_into_ray_tracing_amd/lib/librtmi.so
  for w in nw_motion_blur nw_final; do
    ex=""; [ "$v" = base ] || ex="--no-exec-counts"
    RTMI_LIBRARY=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline $ex > $OUT/${w}_$v.json 2> $OUT/${w}_$v.err || { tail -5 $OUT/${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${w}_$v.json')); r=d['roofline']; print('$w $v', d['value'], r['kernel_ms'], r.get('frac'), r.get('work_equivalent_frac'), r.get('counts'), r.get('note'))"
  done
done
