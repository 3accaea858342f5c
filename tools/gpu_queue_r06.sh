set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06_queue; mkdir -p $OUT
RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_q4s1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_q4s1024.log 2>&1 || { tail -30 $OUT/pytest_q4s1024.log; exit 1; }
tail -2 $OUT/pytest_q4s1024.log
SKIP_TESTS=1 TAG=r06_queue QLIBS="q4s512 q4s1024" timeout -k 10 900 bash tools/gpu_queue.sh
