#!/bin/bash
# Where the grid kernel's HBM writes come from.
# Three rocprofv3 --pmc passes over config 2, each in its own run: store
# instruction counts (scratch spills are flat-scratch stores), the L1->L2
# write requests + WRITE_SIZE, and FETCH_SIZE.  (Round 3 ran it with and
# without the since-removed ramp-down hand-off: profiles/r03/writes/.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-writes}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only $BENCH_ARGS"
for D in $OUT; do
  mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT TA_FLAT_WRITE_WAVEFRONTS_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum --output-format csv -d $D/pmc1 -o pmc1 -- $B > $D/pmc1.json 2> $D/pmc1.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCP_TCC_WRITE_REQ_sum --output-format csv -d $D/pmc2 -o pmc2 -- $B > $D/pmc2.json 2> $D/pmc2.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc3 -o pmc3 -- $B > $D/pmc3.json 2> $D/pmc3.err || exit $?
  python3 tools/pmc_summary.py $D | tee $D/summary.txt
done
