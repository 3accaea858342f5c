#!/bin/bash
# PMC pass (no tracing) on the config-2 bench: LDS and issue counters of the
# render kernel.  BENCH_ARGS, TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmclds_${TAG}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > /dev/null 2> $OUT/pmc1.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > /dev/null 2> $OUT/pmc2.err || exit $?
echo "== $TAG $BENCH_ARGS"
python3 tools/pmc_summary.py $OUT
