"""Analysis: the final scene's layout scaled up (small spheres on a K x K grid
of unit cells, the reference's generator pattern: r = 0.2 at y = 0.2, plus the
ground and the three r = 1 spheres), rendered at 1200x800 with SPP samples
through each closest-hit path: grid (LDS), BVH (LDS when it fits, else walked
in global memory) and brute force.  Prints ms per render (HIP events).
usage: large_scene_bench.py [K ...] (default 22 40 80)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import a_dive_into_ray_tracing_amd as rt  # noqa: E402

W, H, SPP = 1200, 800, int(os.environ.get("SPP", "16"))


def scene(k):
    g = np.random.default_rng(k)
    a, b = np.meshgrid(np.arange(-k // 2, k // 2), np.arange(-k // 2, k // 2))
    n = a.size
    c = np.column_stack([a.ravel() + 0.9 * g.random(n), np.full(n, 0.2), b.ravel() + 0.9 * g.random(n)])
    kinds = np.where(g.random(n) < 0.8, 0, np.where(g.random(n) < 0.75, 1, 2)).astype(np.int32)
    params = np.column_stack([g.random((n, 3)) * g.random((n, 3)), np.where(kinds == 2, 1.5, 0.5 * g.random(n))])
    cr = np.vstack([[0, -1000, 0, 1000], [0, 1, 0, 1], [-4, 1, 0, 1], [4, 1, 0, 1], np.column_stack([c, np.full(n, 0.2)])])
    kinds = np.concatenate([[0, 2, 0, 1], kinds]).astype(np.int32)
    params = np.vstack([[0.5, 0.5, 0.5, 0], [1, 1, 1, 1.5], [0.4, 0.2, 0.1, 0], [0.7, 0.6, 0.5, 0], params])
    return rt.World(cr, kinds, params)


cam = rt.final_camera(W / H)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
st = torch.cuda.Stream()  # (a null handle would mean the context's own stream)
for k in [int(x) for x in sys.argv[1:]] or [22, 40, 80]:
    world = scene(k)
    r = rt.Renderer(world, 0)
    line = [f"{len(world)} spheres:"]
    for accel in ("grid", "bvh", "none"):
        if accel == "none" and len(world) > 3000:
            line.append("none (skipped)")
            continue
        r.set_accel(accel)
        r.render_rows(cam, W, H, SPP, 50, 1984, 0, 1, H, out.data_ptr(), st.cuda_stream)  # cost map
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            r.render_rows(cam, W, H, SPP, 50, 1984, 0, 1, H, out.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        line.append(f"{accel} {e0.elapsed_time(e1) / 3:.2f} ms (path {r.last_schedule()['bvh']})")
    r.close()
    print(" | ".join(line), flush=True)
