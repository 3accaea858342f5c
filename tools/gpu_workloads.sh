#!/bin/bash
# BASELINE configs 4 and 5 on the current tree: the bench
# line of each (roofline with executed-work counts) and a rocprofv3 kernel
# trace of a --timed-only run of the same workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-workloads}
mkdir -p $OUT
for w in ${WORKLOADS:-config4 config5}; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload $w > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['work_equivalent_frac'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$w -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only --workload $w > $OUT/kt_$w.json 2> $OUT/kt_$w.err || { tail -5 $OUT/kt_$w.err; exit 1; }
  find $OUT/kt_$w -name "*kernel_stats.csv" -exec head -3 {} \; | cut -c1-160
  python3 tools/trace_busy.py $(find $OUT/kt_$w -name "*kernel_trace.csv" | head -1) | tee $OUT/kt_${w}_busy.txt
done
