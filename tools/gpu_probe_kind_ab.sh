#!/bin/bash
# The cost probe's kernel: probe_kernel (RTMI_PROBE_KIND=1: 16 pixels of each
# tile, 4 tiles per wave) against a 1-spp render of the rows (0), both to
# depth 8, and probe_kernel to depth 4 and 50: one-shot and steady render
# times of config 2 and one rank's 1/8 strip (tools/oneshot_ab.py), interleaved
# REPS times; then the probe parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-probe_kind}; mkdir -p $OUT
for rep in $(seq ${REPS:-3}); do
  for kd in 0:0 1:0 1:4 1:50; do
    k=${kd%%:*}; d=${kd##*:}
    RTMI_PROBE_KIND=$k RTMI_PROBE_DEPTH=$d timeout -k 10 120 python -u tools/oneshot_ab.py 6 >> $OUT/oneshot.jsonl 2> $OUT/err_${k}_${d}.txt || { tail -5 $OUT/err_${k}_${d}.txt; exit 1; }
    tail -1 $OUT/oneshot.jsonl
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "probe" > $OUT/pytest_probe.log 2>&1 || { tail -30 $OUT/pytest_probe.log; exit 1; }
tail -1 $OUT/pytest_probe.log
