#!/bin/bash
# One-rank RCCL rehearsal of bench.py's N > 1 path on one GPU (RCCL refuses two
# ranks on one device): torch.distributed.run with one rank, backend nccl,
# RTMI_DIST_FORCE=1, so the process group, the async gathers on the CU-masked
# streams, the barriers, the max-over-ranks reductions, the gather check and
# the one-shot gather all run through RCCL.  Then the same with --pipeline 1,
# and the Next-Week bench path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rccl_one_rank}; mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  RTMI_DIST_FORCE=1 NCCL_DEBUG=WARN timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus 1 --no-cpu-baseline "$@" \
    > $OUT/$name.json 2> $OUT/$name.err || { tail -30 $OUT/$name.err; return 1; }
  python - $OUT/$name.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
di, gc, os_ = d.get("dist") or {}, d.get("gather_check"), d.get("one_shot") or {}
print(sys.argv[1], d["value"], d["ms_per_step"], di.get("backend"), di.get("world_size"), di.get("gather_ms_per_rank"),
      gc and gc["bit_exact_vs_1gpu_frame"], os_.get("wall_ms_max_rank"), d.get("one_shot_msamples_per_s"),
      d["config"].get("pipeline"), d["config"].get("dist_rehearsal") is not None)
PY
}
run default --steps 20 --warmup 5 && run p2 --steps 20 --warmup 5 --pipeline 2 && run p1 --steps 10 --warmup 2 --pipeline 1 &&
  run nw --workload nw_motion_blur --nw-spp 50 --steps 3 --warmup 1
