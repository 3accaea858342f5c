#!/bin/bash
# End-of-round check of the current tree (B=<name>): the driver's commands
# (gpu_check.sh with the 1/8 strip), then rocprofv3 kernel traces of the bench
# in both launch modes (--pipeline 2, the default, and --pipeline 1), each with
# the busy time per launch (trace_busy.py).  Outputs under gpurun_out/<B>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-final_check}
TAG=$B STRIP=1 bash tools/gpu_check.sh || exit 1
for p in 2 1; do
  D=gpurun_out/$B/kt_p$p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 bench.py --steps 5 --warmup 1 \
    --no-cpu-baseline --no-exec-counts --timed-only --pipeline $p > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
  python3 -c "import json; r=json.load(open('$D.json'))['roofline']; print('pipeline $p: bench kernel_ms', r['kernel_ms'], 'launch_ms_mean', r['launch_ms_mean'])" | tee $D.txt
  python3 tools/trace_busy.py $(find $D -name "*kernel_trace.csv" | head -1) | tee -a $D.txt
done
