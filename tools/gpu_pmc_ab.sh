#!/bin/bash
# PMC passes (no tracing) over the 1-GPU bench for each kernel shape in
# KERNELS (default "grid resident"), config 2 or BENCH_ARGS: per-dispatch
# means by tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_ab}
mkdir -p $OUT
for k in ${KERNELS:-grid resident}; do
  B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only --pipeline 1 --kernel $k $BENCH_ARGS"
  D=$OUT/$k; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $D/pmc1 -o pmc1 -- $B > $D/pmc1.json 2> $D/pmc1.err || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $D/pmc2 -o pmc2 -- $B > $D/pmc2.json 2> $D/pmc2.err || exit $?
  echo "== $k"; python3 tools/pmc_summary.py $D | tee $D/summary.txt
done
