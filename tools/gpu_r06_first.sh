#!/bin/bash
# Round 6's first GPU pass: the resident kernel (tests + A/B), then the queue
# kernel at 4 waves per SIMD.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r06_resident REPS=2 bash tools/gpu_resident.sh || exit $?
bash tools/gpu_queue_r06.sh
