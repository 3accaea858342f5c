#!/bin/bash
# The driver's round-end commands on the current tree (GPU suite, smoke,
# default bench line), then optional extra steps:
#   TESTS="<pytest args>"  run only these GPU tests (default: tests -m gpu)
#   OLDLIB=<name>  the adversarial-ray tests against lib/librtmi_<name>.so
#                  (a build of an older tree: shows what a fix changed)
#   STRIP=1        the 1/8 strip line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
rm -f gpurun_out/parity_stats.json
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
cp gpurun_out/parity_stats.json $OUT/ 2>/dev/null
tail -1 $OUT/pytest_gpu.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
if [ -n "$STRIP" ]; then
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 > $OUT/strip8.json 2> $OUT/strip8.err || exit 1
  python -c "import json; d=json.load(open('$OUT/strip8.json')); print('strip8', d['roofline']['kernel_ms'])"
fi
if [ -n "$OLDLIB" ]; then
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/librtmi_$OLDLIB.so timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread \
    "tests/test_gpu_parity.py::test_bvh_adversarial_rays_equal_brute_force" "tests/test_gpu_parity.py::test_grid_general_and_one_layer_walks" > $OUT/oldlib_adversarial.log 2>&1
  echo "old library ($OLDLIB) adversarial tests: rc=$?"; tail -3 $OUT/oldlib_adversarial.log
fi
exit 0
