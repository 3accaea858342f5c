set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/oneshot_default; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "probe or cost_probe" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do timeout -k 10 120 python -u tools/oneshot_ab.py 6 | tee -a $OUT/oneshot.jsonl || exit 1; done
