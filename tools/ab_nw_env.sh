#!/bin/bash
# A/B of environment switches (ENVS) on the two Next-Week bench lines (NW_SPP).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for e in ${ENVS:-RTMI_NW_PW=8 RTMI_NW_PW=16}; do
    for w in nw_motion_blur nw_final; do
      env $(echo $e | tr ',' ' ') timeout -k 10 300 python bench.py --workload $w --nw-spp ${NW_SPP:-256} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abnw.json 2> gpurun_out/abnw.err || { tail gpurun_out/abnw.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abnw.json')); print('$e', '$w', $round, d['value'], d['kernel_ms'])"
    done
  done
done
