"""Phase clocks of the queue kernel (analysis only): the RTMI_QUEUE_PHASES
build (lib/librtmi_qph.so, built on the CPU first: python tools/variants.py
build qph; a build from other sources is refused) renders config 2 (or argv W H S) once
through the queue kernel and prints each phase's share of the waves' cycles:
generation, exchange, idle passes, segment (walk + shading), end of segment
(accumulation, next big-sphere pass and key, flushes)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import variants  # noqa: E402

if "RTMI_LIBRARY" not in os.environ:
    why = variants.check("qph")
    if why:
        sys.exit(why)
    os.environ["RTMI_LIBRARY"] = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi_qph.so")
sys.path.insert(0, REPO)
import a_dive_into_ray_tracing_amd as rt  # noqa: E402

W, H, S = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (1200, 800, 500)
L = rt.load()
L.rt_ctx_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
L.rt_ctx_debug_counters.restype = C.c_int
r = rt.Renderer(rt.random_scene(), 0)
r.set_accel("grid")
r.set_kernel("queue")
cam = rt.final_camera(W / H)
r.render(cam, W, H, S, 50, 1984)  # (a first render: cost probe and map)
r.render(cam, W, H, S, 50, 1984)
v = (C.c_uint64 * 8)()
rt.check(L.rt_ctx_debug_counters(r._h, v), "rt_ctx_debug_counters")
names = ["generation", "exchange", "idle passes", "segment (walk + shading)", "end of segment"]
tot = sum(v[1:6])
print(f"{W}x{H}x{S}: world.hit {v[0]}, wave cycles {tot:.4g}")
for k, n in enumerate(names):
    print(f"  {n:28s} {v[1 + k] / tot:.3f}")
