#!/bin/bash
# One rank's strip of an N-GPU config-2 render (N = 2, 4) over item sizes whose
# items per tile stay a multiple of 4 (block flush); kernel ms.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/snc
run() {
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/snc/s.json 2> gpurun_out/snc/s.err || { tail gpurun_out/snc/s.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/snc/s.json')); print(sys.argv[1:], d['roofline']['kernel_ms'])" "$@"
}
for n in 4 2; do
  run --strip-of $n
  for ch in 25 42 63 125; do run --strip-of $n --chunk $ch; done
done
