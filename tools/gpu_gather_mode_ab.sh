#!/bin/bash
# Where the timed steps' gathers run (bench.py's N > 1 path as a one-rank RCCL
# run, RTMI_DIST_FORCE=1): async on torch's NCCL stream ("side", with the
# default 4 hardware queues; round 6 also ran it with 8) against synchronous on the render's own
# stream over a process group per context ("inline"), frame and 1/8 strip, interleaved REPS times, with the plain
# single-GPU line beside them.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gather_mode}; mkdir -p $OUT
STEPS=${STEPS:-20}
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus 1 --no-cpu-baseline --no-exec-counts \
    --timed-only --steps $STEPS --warmup 5 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -30 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().splitlines()[-1]); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], r['launch_ms_mean'], (d.get('dist') or {}).get('gather_ms_per_rank'))" | tee -a $OUT/ab.txt
}
for rep in $(seq ${REPS:-2}); do
  for so in 1 8; do
    sa=""; [ $so -gt 1 ] && sa="--strip-of $so"
    one plain_s${so}_$rep RTMI_DIST_FORCE=0 -- $sa || exit 1
    one side_s${so}_$rep RTMI_DIST_FORCE=1 -- $sa || exit 1
    one inline_s${so}_$rep RTMI_DIST_FORCE=1 RTMI_BENCH_GATHER=inline -- $sa || exit 1
  done
done
