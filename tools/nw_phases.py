"""Phase split of the Next-Week kernel (RTMI_NW_PHASES build, run on the GPU box;
built on the CPU first: python tools/variants.py build nwph — a build from
other sources is refused)
Prints, per scene and structure, the share of a wave's item time in the closest
hit, in hit record + texture + scatter, and in accumulation + regeneration."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import variants  # noqa: E402

if variants.check("nwph"):
    sys.exit(variants.check("nwph"))
os.environ["RTMI_LIBRARY"] = os.path.join(ROOT, "a_dive_into_ray_tracing_amd", "lib", "librtmi_nwph.so")
import torch  # noqa: E402,F401  (one HIP runtime)
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402
from a_dive_into_ray_tracing_amd._abi import load  # noqa: E402

L = load()
L.rt_nw_debug_phases.argtypes = [C.POINTER(C.c_uint64)]
earth = nw.load_image(os.path.join(ROOT, "tests", "golden", "earthmap.jpeg"))
for which, W, H, spp in ((1, 1200, 800, 64), (8, 800, 800, 64)):
    s, cam = nw.preset(which, image=earth, aspect=W / H)
    for accel in ("bvh", "grid"):
        r = nw.NwRenderer(s)
        r.set_accel(accel)
        used = r.accel_info()["accel"]
        r.render(cam, W, H, spp, 50, 1984)
        out = (C.c_uint64 * 4)()
        L.rt_nw_debug_phases(out)  # discard the first render's
        import time
        t0 = time.time()
        r.render(cam, W, H, spp, 50, 1984)
        dt = time.time() - t0
        L.rt_nw_debug_phases(out)
        v = np.array(list(out), dtype=np.float64)
        print(f"scene {which} {W}x{H}x{spp} {accel}->{used}: {dt * 1e3:.1f} ms; hit {v[0] / v[3]:.3f}, "
              f"record+texture+scatter {v[1] / v[3]:.3f}, accumulate+regenerate {v[2] / v[3]:.3f}", flush=True)
        r.close()
