#!/bin/bash
# Interleaved A/B of bench configurations: CFGS holds ';'-separated
# "ENV=v ...|bench arguments" sets (each run on config 2 and, with STRIP=1, one rank's 1/8
# strip), REPS repetitions.  Lines "rep | args | strip | ms_per_step
# kernel_ms" in gpurun_out/$TAG/ab.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_cfgs}
mkdir -p $OUT
B="--steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only"
IFS=';' read -ra LIST <<< "$CFGS"
for rep in $(seq ${REPS:-2}); do
  for cfg in "${LIST[@]}"; do
    for strip in ${STRIPS:-0 8}; do
      sa=""; [ $strip -gt 0 ] && sa="--strip-of $strip"
      envs=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 120 env $envs python -u bench.py $B $args $sa > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/b.json')); print('$rep |', '$cfg', '| strip=$strip |', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
