cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/q && LIBS="old base" TAG=ab_med3 bash tools/gpu_ab_lib.sh
