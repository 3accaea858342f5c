#!/bin/bash
# Next-Week parity suite, then both Next-Week workloads at 256 spp and full spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nwa
timeout -k 10 300 python -u -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/nwa/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/nwa/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in nw_motion_blur nw_final; do
  for spp in 256 0; do
    a=""; [ $spp -gt 0 ] && a="--nw-spp $spp"
    timeout -k 10 200 python bench.py --workload $w $a --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nwa/$w$spp.json 2> gpurun_out/nwa/e.err || { tail gpurun_out/nwa/e.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nwa/$w$spp.json')); print('$w', '$a', d['ms_per_step'], d['value'])"
  done
done
