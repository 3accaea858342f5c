#!/bin/bash
# bench rework check: default bench line (exec counts + CPU baseline rows),
# the N>1 launcher rehearsed with gloo (ranks share the one GPU), and a
# refusal of --gpus 2 under nccl on a 1-GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r2b
mkdir -p $OUT
echo "== bench" && timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== refuse" ; timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > $OUT/refuse.out 2>&1; echo "rc=$?"; tail -2 $OUT/refuse.out
echo "== gloo 2" && RTMI_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --no-cpu-baseline --no-exec-counts > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail $OUT/gloo2.err; exit 1; }
cat $OUT/gloo2.json
echo "== gloo 4" && RTMI_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 --steps 2 --no-cpu-baseline > $OUT/gloo4.json 2> $OUT/gloo4.err || { tail $OUT/gloo4.err; exit 1; }
cat $OUT/gloo4.json
