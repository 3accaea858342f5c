#!/bin/bash
# Misc measurements on the current tree: persistent vs grid kernel on the 1/8
# strip (grid accel), configs 4 and 5 bench lines, HBM traffic of the grid
# kernel (FETCH_SIZE / WRITE_SIZE in separate PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-misc}
mkdir -p $OUT
for k in grid persistent; do
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-exec-counts --timed-only --strip-of 8 --kernel $k > $OUT/s8_$k.json 2> $OUT/s8_$k.err || exit 1
  python -c "import json; d=json.load(open('$OUT/s8_$k.json')); print('strip8 kernel $k', d['roofline']['kernel_ms'])"
done
for w in config4 config5; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload $w > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['work_equivalent_frac'])"
done
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exec-counts --timed-only"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o pmc1 -- $B > $OUT/pmc1.json 2> $OUT/pmc1.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o pmc2 -- $B > $OUT/pmc2.json 2> $OUT/pmc2.err || exit 1
python3 tools/pmc_summary.py $OUT | tee $OUT/traffic_summary.txt
