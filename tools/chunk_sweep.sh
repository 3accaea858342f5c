#!/bin/bash
# Config-2 bench at several first-phase chunk sizes (CHUNKS), default library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in ${CHUNKS:-50 63 32 125}; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --chunk $c $BENCH_ARGS > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/chunk_$c.json')); print('chunk', $c, d['value'], d['roofline']['kernel_ms'])"
done
