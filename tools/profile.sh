#!/bin/bash
# rocprofv3 passes over the 1-GPU bench (config 2).  Kernel trace + stats in
# one pass; PMC counters in their own passes (never mixed with tracing).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt_bench.json 2> $OUT/kt.err || exit $?
echo "== pmc 1"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > /dev/null 2> $OUT/pmc1.err || exit $?
echo "== pmc 2"
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > /dev/null 2> $OUT/pmc2.err || exit $?
echo "== pmc 5"
timeout -k 10 600 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_INST_LEVEL_SMEM SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 SQ_CYCLES SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $OUT/pmc5 -o pmc5 -- $B > /dev/null 2> $OUT/pmc5.err || exit $?
echo "== pmc hbm read"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o pmc3 -- $B > /dev/null 2> $OUT/pmc3.err || exit $?
echo "== pmc hbm write"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o pmc4 -- $B > /dev/null 2> $OUT/pmc4.err || exit $?
find $OUT -name "*.csv" | head -20
