#!/bin/bash
# rocprofv3 passes over the 1-GPU bench (config 2; BENCH_ARGS adds e.g.
# "--accel grid").  Kernel trace + stats in one pass; PMC counters in their own
# passes (never mixed with tracing), each within the per-block limits.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof_r02}
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only $BENCH_ARGS"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt_bench.json 2> $OUT/kt.err || exit $?
echo "== pmc 1"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > /dev/null 2> $OUT/pmc1.err || exit $?
echo "== pmc 2"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > /dev/null 2> $OUT/pmc2.err || exit $?
echo "== pmc 3"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_CYCLES --output-format csv -d $OUT/pmc3 -o pmc3 -- $B > /dev/null 2> $OUT/pmc3.err || exit $?
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
