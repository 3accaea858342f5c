"""Engine comparison (GPU box): the RTIOW final scene rendered by the Next-Week
kernel (NW builder: spheres + lambertian/metal/dielectric, shutter [0, 0])
against the RTIOW kernel, config-2 size at a reduced spp; and the Next-Week
motion-blur scene with its shutter closed.  Prints Msamples/s and world.hit/s."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime)
import a_dive_into_ray_tracing_amd as rt  # noqa: E402
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402

W, H, S = 1200, 800, int(sys.argv[1]) if len(sys.argv) > 1 else 64
world = rt.random_scene()
s = nw.Scene()
for k in range(len(world)):
    c, r = world.center_radius[k, :3], world.center_radius[k, 3]
    kind, p = int(world.mat_kind[k]), world.mat_params[k]
    if kind == 0:
        m = s.lambertian(s.solid(*p[:3]))
    elif kind == 1:
        m = s.metal(s.solid(*p[:3]), min(p[3], 1.0))
    else:
        m = s.dielectric(p[3])
    s.add(s.sphere(tuple(c), r, m))
s.set_background(0.7, 0.8, 1.0)


def timed(fn, reps=2):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


cam = nw.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, W / H, 0.1, 10.0, 0.0, 0.0)
r = nw.NwRenderer(s)
dt = timed(lambda: r.render(cam, W, H, S, 50, 1984))
segs = r.last_segments()
print(f"NW kernel on the RTIOW scene: {W * H * S / dt / 1e6:.0f} Msamples/s, {segs / dt / 1e9:.2f} G world.hit/s, "
      f"{segs / (W * H * S):.3f} segs/sample, info {r.info()}")
r.close()
rr = rt.Renderer(world, 0)
rr.set_accel("bvh")
cam2 = rt.final_camera(W / H)
dt = timed(lambda: rr.render(cam2, W, H, S, 50, 1984))
segs = rr.last_segments()
print(f"RTIOW kernel: {W * H * S / dt / 1e6:.0f} Msamples/s, {segs / dt / 1e9:.2f} G world.hit/s")
rr.close()
mb, mcam = nw.preset(1, aspect=W / H)
for shutter in ((0.0, 1.0), (0.0, 0.0)):
    cam3 = nw.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, W / H, 0.1, 10.0, *shutter)
    r = nw.NwRenderer(mb)
    dt = timed(lambda: r.render(cam3, W, H, S, 50, 1984))
    segs = r.last_segments()
    print(f"NW motion-blur scene, shutter {shutter}: {W * H * S / dt / 1e6:.0f} Msamples/s, {segs / dt / 1e9:.2f} G world.hit/s")
    r.close()
