#!/bin/bash
# A/B of bench.py --pipeline 1 / 2 on config 2 (frame, strips of 2 / 4 / 8)
# and config 5's strip of 8, REPS alternating repetitions; one summary line
# per run into $OUT/ab.txt.
set -e -o pipefail
OUT=${OUT:-gpurun_out/pipeline}
REPS=${REPS:-2}
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for p in 1 2; do
    for n in 1 2 4 8; do
      steps=$((10 * n)); [ "$n" = 1 ] && steps=10
      so=""; [ "$n" -gt 1 ] && so="--strip-of $n"
      timeout -k 10 300 python -u bench.py --steps "$steps" --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only \
        --pipeline "$p" $so > "$OUT/c2_n${n}_p${p}_$rep.json"
      python -c "import json; d=json.load(open('$OUT/c2_n${n}_p${p}_$rep.json')); r=d['roofline']; print('config2 1/$n pipeline $p rep $rep: ms_per_step', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'launch_ms_mean', r['launch_ms_mean'], 'value', d['value'])" | tee -a "$OUT/ab.txt"
    done
    if [ -n "$C5" ]; then
      timeout -k 10 300 python -u bench.py --workload config5 --steps 6 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only \
        --pipeline "$p" --strip-of 8 > "$OUT/c5_n8_p${p}_$rep.json"
      python -c "import json; d=json.load(open('$OUT/c5_n8_p${p}_$rep.json')); r=d['roofline']; print('config5 1/8 pipeline $p rep $rep: ms_per_step', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'launch_ms_mean', r['launch_ms_mean'])" | tee -a "$OUT/ab.txt"
    fi
  done
done
