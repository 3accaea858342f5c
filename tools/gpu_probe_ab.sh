#!/bin/bash
# One-shot render A/B: the cost probe's samples per pixel (RTMI_PROBE_SPP;
# 0 = the library's automatic choice), twice each, interleaved: bench.py's
# one_shot (probe pass + cost-ordered render, HIP events) on config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probe_ab}
mkdir -p $OUT
for rep in 1 2; do
  for ps in ${PROBES:-0 1}; do
    RTMI_PROBE_SPP=$ps timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/p${ps}_$rep.json 2> $OUT/p${ps}_$rep.err || { tail -3 $OUT/p${ps}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p${ps}_$rep.json')); print('probe_spp $ps', d['roofline']['kernel_ms'], d['one_shot'])"
  done
done
