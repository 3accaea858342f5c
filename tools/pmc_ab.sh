#!/bin/bash
# PMC passes 1-2 (no tracing) for one bench configuration: BENCH_ARGS, TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcab_${TAG}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > /dev/null 2> $OUT/pmc1.err || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > /dev/null 2> $OUT/pmc2.err || exit $?
echo "== $TAG $BENCH_ARGS"
python3 tools/pmc_summary.py $OUT
