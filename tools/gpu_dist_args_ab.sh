#!/bin/bash
# A/B of bench.py argument sets through the N > 1 path as a one-rank RCCL run
# (RTMI_DIST_FORCE=1; ARGSETS="a|b|...", each set may start with VAR=value
# environment words), REPS (2) times each, interleaved, STEPS (20) timed steps:
# ms per step, busy ms per launch, mean launch ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dist_args_ab}; mkdir -p $OUT
IFS='|' read -r -a SETS <<< "$ARGSETS"
for rep in $(seq 1 "${REPS:-2}"); do
  for i in "${!SETS[@]}"; do
    envs=(RTMI_DIST_FORCE=1); args=()
    for w in ${SETS[$i]}; do if [[ ${#args[@]} -eq 0 && $w == *=* && $w != -* ]]; then envs+=("$w"); else args+=("$w"); fi; done
    env "${envs[@]}" timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
      --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus 1 --no-cpu-baseline --no-exec-counts \
      --timed-only --steps ${STEPS:-20} --warmup 5 "${args[@]}" > $OUT/set${i}_$rep.json 2> $OUT/set${i}_$rep.err \
      || { tail -20 $OUT/set${i}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/set${i}_$rep.json').read().splitlines()[-1]); r=d['roofline']; print('[${SETS[$i]}]', d['ms_per_step'], r['kernel_ms'], r['launch_ms_mean'])" | tee -a $OUT/ab.txt
  done
done
