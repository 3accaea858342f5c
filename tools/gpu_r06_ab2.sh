set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06_ab_res REPS=2 AB="grid:grid:- res:resident:- rw8:resident:rw8 rnf:resident:rnf rst:resident:rst" bash tools/gpu_ab_kernels.sh || exit $?
TAG=r06_ab_queue REPS=1 AB="grid:grid:- queue:queue:- q4s512:queue:q4s512 q4s1024:queue:q4s1024" bash tools/gpu_ab_kernels.sh
