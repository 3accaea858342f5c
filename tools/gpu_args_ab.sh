#!/bin/bash
# A/B of bench.py argument sets on config 2 (ARGSETS="a|b|..." — e.g.
# "--tile-w 8|--tile-w 16"), REPS (2) times each, interleaved, STEPS (10)
# timed steps per run: kernel ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-args_ab}
mkdir -p $OUT
IFS='|' read -r -a SETS <<< "$ARGSETS"
for rep in $(seq 1 "${REPS:-2}"); do
  for i in "${!SETS[@]}"; do
    timeout -k 10 150 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only ${SETS[$i]} > $OUT/set${i}_$rep.json 2> $OUT/set${i}_$rep.err || { tail -3 $OUT/set${i}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/set${i}_$rep.json')); print('[${SETS[$i]}]', d['roofline']['kernel_ms'], d['config']['tile'])" | tee -a $OUT/ab.txt
  done
done
