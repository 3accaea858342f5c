#!/bin/bash
# A/B of environment settings (ENVSETS="A=1|A=2 B=3|..."; "" = none) on config 2
# and one rank's strips (STRIPS="1 8": 1 = the frame, N = --strip-of N), REPS
# (2) times, interleaved, STEPS (10) timed steps per run: kernel ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-env_ab}
mkdir -p $OUT
IFS='|' read -r -a SETS <<< "$ENVSETS"
for rep in $(seq 1 "${REPS:-2}"); do
  for i in "${!SETS[@]}"; do
    line="[${SETS[$i]}]"
    for n in ${STRIPS:-1 8}; do
      so=""; [ "$n" -gt 1 ] && so="--strip-of $n"
      env ${SETS[$i]} timeout -k 10 150 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts \
        --timed-only $so $BENCH_ARGS > $OUT/set${i}_n${n}_$rep.json 2> $OUT/set${i}_n${n}_$rep.err || { tail -3 $OUT/set${i}_n${n}_$rep.err; exit 1; }
      line="$line 1/$n $(python -c "import json; print(json.load(open('$OUT/set${i}_n${n}_$rep.json'))['roofline']['kernel_ms'])")"
    done
    echo "$line" | tee -a $OUT/ab.txt
  done
done
