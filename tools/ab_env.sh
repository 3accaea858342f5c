#!/bin/bash
# A/B of environment switches (ENVS, space-separated NAME=VALUE sets joined by
# commas) on the config-2 bench and one rank's 1/8 strip, interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for e in ${ENVS:-RTMI_DYN_ITEMS=1 RTMI_DYN_ITEMS=0}; do
    for args in "" "--strip-of 8"; do
      env $(echo $e | tr ',' ' ') timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $args $BENCH_ARGS > gpurun_out/abenv.json 2> gpurun_out/abenv.err || { tail gpurun_out/abenv.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abenv.json')); print('$e', '$args', $round, d['value'], d['roofline']['kernel_ms'])"
    done
  done
done
