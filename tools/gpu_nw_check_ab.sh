cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/nw_boxinv && timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/nw_boxinv/pytest.log 2>&1 || { tail -30 gpurun_out/nw_boxinv/pytest.log; exit 1; }
tail -2 gpurun_out/nw_boxinv/pytest.log
LIBS="base nwold" TAG=ab_nw_boxinv bash tools/gpu_ab_nw_lib.sh
