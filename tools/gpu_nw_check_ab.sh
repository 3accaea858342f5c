#!/bin/bash
# Next-Week parity tests, then an A/B of librtmi.so against librtmi_nwold.so (tools/gpu_ab_nw_lib.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-nw_check}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
LIBS="base nwold" TAG=ab_$T bash tools/gpu_ab_nw_lib.sh
