"""BVH / grid walk statistics of the RTMI_STATS build at config 2 (GPU box).
    python tools/bvh_stats.py [bvh|grid]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["RTMI_LIBRARY"] = os.path.join(ROOT, "a_dive_into_ray_tracing_amd", "lib", "librtmi_stats.so")
import a_dive_into_ray_tracing_amd as rt  # noqa: E402

L = rt.load()
L.rt_ctx_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
r = rt.Renderer(rt.random_scene(), 0)
accel = sys.argv[1] if len(sys.argv) > 1 else "bvh"
r.set_accel(accel)
print(accel, "accel info:", r.accel_info() if accel == "bvh" else r.grid_info())
r.render(rt.final_camera(1.5), 1200, 800, 500, 50, 1984)
v = (C.c_uint64 * 8)()
L.rt_ctx_debug_counters(r._h, v)
segs = v[0]
print(f"segments {segs}; per lane-segment: node visits {v[5] / segs:.2f}, leaf sphere tests {v[6] / segs:.2f}, "
      f"resolves {v[3] / segs:.2f}")
ws = segs / 64.0  # wave-segments (lane utilisation ~0.997)
print(f"per wave-segment: node iterations {v[1] / ws:.2f}, leaf-sphere iterations {v[2] / ws:.2f}, "
      f"root-resolution blocks {v[4] / ws:.2f}")
