#!/bin/bash
# The second record call: the N>1 rehearsal through bench.py's own
# launcher (gloo, N ranks on one GPU), HBM traffic of the BVH and brute-force
# kernels on the current tree, their
# bench lines, and the walk counters + phase clocks (gpu_phases.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-extras}
mkdir -p gpurun_out/$B
TAG=$B/gloo RANKS="2 3 8" bash tools/gpu_gloo_rehearsal.sh || exit 1
for acc in bvh none; do
  TAG=$B/traffic_$acc BENCH_ARGS="--accel $acc" bash tools/pmc_traffic.sh > gpurun_out/$B/traffic_$acc.log 2>&1 || { tail -5 gpurun_out/$B/traffic_$acc.log; exit 1; }
  timeout -k 10 300 python -u bench.py --accel $acc --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$B/$acc.json 2> gpurun_out/$B/$acc.err || { tail -5 gpurun_out/$B/$acc.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$B/$acc.json')); r=d['roofline']; print('$acc', d['value'], r['kernel_ms'], r['frac'], r['work_equivalent_frac'])"
done
TAG=$B/phases bash tools/gpu_phases.sh || exit 1
