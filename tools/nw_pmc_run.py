"""The RTIOW final scene through the Next-Week kernel (for rocprofv3 --pmc):
one warm-up and one measured render at 1200x800 and argv[1] spp; prints
world.hit calls of the last render."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import a_dive_into_ray_tracing_amd as rt  # noqa: E402
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402

W, H, S = 1200, 800, int(sys.argv[1]) if len(sys.argv) > 1 else 64
world = rt.random_scene()
s = nw.Scene()
for k in range(len(world)):
    c, r = world.center_radius[k, :3], world.center_radius[k, 3]
    kind, p = int(world.mat_kind[k]), world.mat_params[k]
    m = s.lambertian(s.solid(*p[:3])) if kind == 0 else s.metal(s.solid(*p[:3]), min(p[3], 1.0)) if kind == 1 else s.dielectric(p[3])
    s.add(s.sphere(tuple(c), r, m))
s.set_background(0.7, 0.8, 1.0)
cam = nw.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, W / H, 0.1, 10.0, 0.0, 0.0)
r = nw.NwRenderer(s)
for _ in range(2):
    r.render(cam, W, H, S, 50, 1984)
print("segments", r.last_segments())
r.close()
