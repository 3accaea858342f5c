#!/bin/bash
# The resident grid kernel (experimental build) with a short-item tail phase:
# its waves never leave, so a launch ends when each wave's last item does (the
# per-wave trace: frame waves end between 18.6 and 20.0 ms).  Config 2 frame
# and one rank's 1/8 strip, single launches; SETS="name|bench args;..." run
# against the grid kernel of the product library, REPS times interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-resident_tail}; mkdir -p $OUT
EXP=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_experimental.so
run() {  # name, lib (- = product), bench args...
  local name=$1 lib=$2; shift 2
  local L=""; [ "$lib" != "-" ] && L=$EXP
  RTMI_LIBRARY=$L timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-exec-counts \
    --timed-only --pipeline 1 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
}
IFS=';' read -r -a S <<< "${SETS:-grid|--kernel grid;res|--kernel resident;res_t50c5|--kernel resident --tail-spp 50 --tail-chunk 5;res_t100c10|--kernel resident --tail-spp 100 --tail-chunk 10;res_t25c2|--kernel resident --tail-spp 25 --tail-chunk 2}"
for rep in $(seq ${REPS:-2}); do
  for so in 1 8; do
    for spec in "${S[@]}"; do
      name=${spec%%|*}; args=${spec#*|}
      lib=-; [[ $args == *resident* ]] && lib=exp
      sa=""; [ $so -gt 1 ] && sa="--strip-of $so"
      run ${name}_s${so}_$rep $lib $args $sa || exit 1
    done
  done
done
