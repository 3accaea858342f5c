#!/bin/bash
# Kernel-level strong-scaling ceiling: one rank's
# interleaved 1/N strip (bench.py --strip-of N) against the whole frame on one
# GPU, N = 2, 4, 8, for config 2 and config 5.  A ceiling, not a scaling
# measurement: no gather, no launch skew, one GPU.  Table in $OUT/strips.txt.
# PIPELINE (default 1: one context, one launch at a time, as the round-5 table
# in profiles/r05/strips/; 2: bench.py's default, steps overlapping).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-strips}
mkdir -p $OUT
for w in config2 config5; do
  steps=10; [ $w = config5 ] && steps=3
  for n in 1 2 4 8; do
    so=""; [ $n -gt 1 ] && so="--strip-of $n"
    timeout -k 10 300 python -u bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline --no-exec-counts \
      --timed-only --pipeline ${PIPELINE:-1} $so > $OUT/${w}_$n.json 2> $OUT/${w}_$n.err || { tail $OUT/${w}_$n.err; exit 1; }
    echo "$w 1/$n $(python -c "import json; print(json.load(open('$OUT/${w}_$n.json'))['roofline']['kernel_ms'])")"
  done
done
python - "$OUT" > $OUT/strips.txt <<'PY'
import json, sys
out = sys.argv[1]
print("# one rank's interleaved 1/N strip vs the frame (kernel ms, HIP events; bench.py --strip-of N), one GPU")
print("# efficiency = frame / (N x strip): the kernel-level strong-scaling ceiling before gather and launch overheads")
print(f"{'workload':10s} {'N':>2s} {'kernel_ms':>10s} {'ideal_ms':>9s} {'efficiency':>10s} {'ceiling_x':>9s}")
for w in ("config2", "config5"):
    f = json.load(open(f"{out}/{w}_1.json"))["roofline"]["kernel_ms"]
    for n in (1, 2, 4, 8):
        k = json.load(open(f"{out}/{w}_{n}.json"))["roofline"]["kernel_ms"]
        print(f"{w:10s} {n:2d} {k:10.3f} {f / n:9.3f} {f / (n * k):10.3f} {f / k:9.2f}")
PY
cat $OUT/strips.txt
