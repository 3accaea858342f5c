"""Debug aid for the queue kernel (analysis only): render one configuration
through the grid kernel and the queue kernel several times and print where
and by how much they differ (usage: queue_debug.py W H S tile_w [probe])."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import a_dive_into_ray_tracing_amd as rt  # noqa: E402

W, H, S, TW = (int(x) for x in sys.argv[1:5])
world = rt.random_scene()
cam = rt.final_camera(W / H)
g = rt.Renderer(world, 0)
g.set_accel("grid")
ref = g.render(cam, W, H, S, 50, 1984)
q = rt.Renderer(world, 0)
q.set_accel("grid")
q.set_kernel("queue")
q.set_tuning(TW, 0)
for it in range(4):
    img = q.render(cam, W, H, S, 50, 1984)
    d = np.abs(img - ref).max(axis=2)
    bad = np.argwhere(d > 0)
    print(f"run {it}: schedule {q.last_schedule()} segs {q.last_segments()} vs {g.last_segments()}; "
          f"{len(bad)} pixels differ, max {d.max():.4f}", flush=True)
    for j, i in bad[:12]:
        print(f"   pixel (row {j}, col {i}) tile ({i // TW}, {j // (64 // TW)}): queue {img[j, i]} grid {ref[j, i]}")
