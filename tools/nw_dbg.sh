cd "$GRAFT_REPO_ROOT"
for lib in librtmi.so librtmi_p_noobj.so librtmi_g_obj.so librtmi_g_noobj.so; do
  RTMI_LIBRARY=$PWD/a_dive_into_ray_tracing_amd/lib/$lib timeout -k 10 120 python -m pytest tests/test_nw_gpu.py -q -k "bit_exact_vs_oracle" --timeout 100 2>&1 | tail -2 | head -1 | sed "s/^/$lib: /"
done
