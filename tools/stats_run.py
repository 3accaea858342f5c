"""Debug counters of the RTMI_STATS build at config 2 (run on the GPU box)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["RTMI_LIBRARY"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "a_dive_into_ray_tracing_amd", "lib", "librtmi_stats.so")
import a_dive_into_ray_tracing_amd as rt

L = rt.load()
L.rt_ctx_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
r = rt.Renderer(rt.random_scene(), 0)
r.render(rt.final_camera(1.5), 1200, 800, 500, 50, 1984)
v = (C.c_uint64 * 8)()
L.rt_ctx_debug_counters(r._h, v)
segs, groups, any_groups, resolves, wave_sph = list(v)[:5]
wseg = groups / 61
print(f"per wave-segment: groups-with-candidate {any_groups / wseg:.2f}, spheres resolved (wave) {wave_sph / wseg:.2f}, "
      f"lane resolves per lane-segment {resolves / segs:.2f}")
print(f"segments {segs} groups {groups} groups_with_candidate {any_groups} ({any_groups / groups:.3f}) "
      f"lane_resolves {resolves} (per lane-segment {resolves / segs:.2f}; per sphere-test {resolves / (segs * 487):.4f}); "
      f"wave-segments {wseg:.4g}; lane utilisation {segs / (wseg * 64):.3f}")
