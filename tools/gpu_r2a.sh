#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2a
mkdir -p $OUT
echo "== smoke" && timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo "== bench" && timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== stats" && timeout -k 10 200 python -u tools/bvh_stats.py > $OUT/bvh_stats.txt 2>&1 || { tail $OUT/bvh_stats.txt; exit 1; }
cat $OUT/bvh_stats.txt
nproc; lscpu | head -30 > $OUT/lscpu.txt; cat $OUT/lscpu.txt; numactl -H 2>/dev/null | head -5; which taskset numactl
