#!/bin/bash
# A/B of the product library against a variant build (VARIANT=name, built on
# the CPU by tools/variants.py): config 2 frame and one rank's 1/8 strip,
# --pipeline 1 and 2, REPS times interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
V=${VARIANT:?VARIANT=name}
python tools/variants.py check $V || exit 1
OUT=gpurun_out/${TAG:-variant_ab}; mkdir -p $OUT
VL=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$V.so
run() {  # name, lib, bench args...
  local name=$1 lib=$2; shift 2
  RTMI_LIBRARY=$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    --no-exec-counts --timed-only "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
}
for rep in $(seq ${REPS:-2}); do
  for p in 1 2; do
    for so in 1 8; do
      sa=""; [ $so -gt 1 ] && sa="--strip-of $so"
      run product_p${p}_s${so}_$rep "" --pipeline $p $sa || exit 1
      run ${V}_p${p}_s${so}_$rep $VL --pipeline $p $sa || exit 1
    done
  done
done
