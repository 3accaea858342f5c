#!/bin/bash
# One-shot render time against the cost probe's depth limit and samples
# (tools/oneshot_ab.py per setting, interleaved twice).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-oneshot_ab}; mkdir -p $OUT
for rep in 1 2; do
  for d in 0 8 4 2; do
    for sp in 0 1; do
      RTMI_PROBE_DEPTH=$d RTMI_PROBE_SPP=$sp timeout -k 10 120 python -u tools/oneshot_ab.py 6 >> $OUT/oneshot.jsonl 2> $OUT/err_${d}_${sp}.txt || { tail -5 $OUT/err_${d}_${sp}.txt; exit 1; }
      tail -1 $OUT/oneshot.jsonl
    done
  done
done
