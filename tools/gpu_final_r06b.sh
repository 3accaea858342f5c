#!/bin/bash
# Round 6 final record, part B (B=<name>, default r06_final): configs 4 and 5
# (gpu_workloads.sh), a rocprofv3 kernel trace with --pipeline 1, and the
# end-to-end rates (tools/end_to_end.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-r06_final}
mkdir -p gpurun_out/$B
TAG=$B/workloads bash tools/gpu_workloads.sh || exit 1
D=gpurun_out/$B/kt_p1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 bench.py --steps 5 --warmup 1 \
  --no-cpu-baseline --no-exec-counts --timed-only --pipeline 1 > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
python3 -c "import json; r=json.load(open('$D.json'))['roofline']; print('pipeline 1: bench kernel_ms', r['kernel_ms'])" | tee $D.txt
python3 tools/trace_busy.py $(find $D -name "*kernel_trace.csv" | head -1) | tee -a $D.txt
timeout -k 10 300 python3 -u tools/end_to_end.py > gpurun_out/$B/e2e.json 2> gpurun_out/$B/e2e.err || { tail -5 gpurun_out/$B/e2e.err; exit 1; }
cat gpurun_out/$B/e2e.json
