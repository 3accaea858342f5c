#!/bin/bash
# Where the resident kernel's extra wait cycles go: one PMC pass
# of wait / active-instruction counters for the grid and resident kernels
# (experimental library), config 2, single launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_ab2}; mkdir -p $OUT
export RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_experimental.so
for k in grid resident; do
  D=$OUT/$k; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $D/pmc1 -o pmc1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only --pipeline 1 --kernel $k > $D/pmc1.json 2> $D/pmc1.err || { tail -5 $D/pmc1.err; exit 1; }
  echo "== $k"; python3 tools/pmc_summary.py $D | tee $D/summary.txt
done
