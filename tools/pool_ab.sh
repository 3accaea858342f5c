#!/bin/bash
# Block-shared job pool A/B: parity of the pool variants, then config 2 and one
# rank's 1/8 strip with RTMI_BLOCK_POOL=0/1, then the strip over chunk sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-pool}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "block_flush" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pool in 0 1; do
  for args in "" "--strip-of 8" "--strip-of 8 --tile-w 16"; do
    RTMI_BLOCK_POOL=$pool timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $args > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b.json')); print('pool', $pool, '$args', d['roofline']['kernel_ms'])"
  done
done
for tw in 8 16; do
  for ch in ${CHUNKS:-7 9 14 18 21}; do
    timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --strip-of 8 --tile-w $tw --chunk $ch > $OUT/s.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/s.json')); print('strip tile_w', $tw, 'chunk', $ch, d['roofline']['kernel_ms'])"
  done
done
for ch in 21 25 32 42 63; do
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --chunk $ch > $OUT/s.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s.json')); print('frame chunk', $ch, d['roofline']['kernel_ms'])"
done
