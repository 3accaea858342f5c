cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/nwpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/nwpmc/pmc1 -o pmc1 -- python3 tools/nw_pmc_run.py 64 > gpurun_out/nwpmc/run1.txt 2> gpurun_out/nwpmc/pmc1.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_FLOPS_FP32 --output-format csv -d gpurun_out/nwpmc/pmc2 -o pmc2 -- python3 tools/nw_pmc_run.py 64 > gpurun_out/nwpmc/run2.txt 2> gpurun_out/nwpmc/pmc2.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nwpmc/kt -o kt -- python3 tools/nw_pmc_run.py 64 > gpurun_out/nwpmc/run3.txt 2> gpurun_out/nwpmc/kt.err || exit 1
cat gpurun_out/nwpmc/run1.txt
