cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in librtmi.so librtmi_p6.so; do
 for args in "--kernel grid --strip-of 8" "--kernel persistent --strip-of 8" "--kernel persistent"; do
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/p6.json 2>gpurun_out/p6.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/p6.json')); print('$lib', '$args', d['roofline']['kernel_ms'])"
 done
done
