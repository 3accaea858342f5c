#!/bin/bash
# A/B kernel variants (librtmi_<name>.so), each in its own process, interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"librtmi.so"}
for round in 1 2; do
  for lib in $VARIANTS; do
    RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_${lib}_$round.json 2>gpurun_out/ab_${lib}_$round.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${lib}_$round.json')); print('$lib', $round, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
