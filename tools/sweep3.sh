#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
IFS=","; for args in ${SWEEP}; do unset IFS;
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/sweep.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('gpurun_out/sweep.json')); print('$args', d['value'], d['roofline']['kernel_ms'])"
done
