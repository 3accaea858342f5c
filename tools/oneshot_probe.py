"""Analysis: K one-shot renders of config 2 (each forgets the cost map, so it
runs the probe pass first) on one context; prints each render's wall ms.
Run under rocprofv3 --kernel-trace to split the probe, main and finalize."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import a_dive_into_ray_tracing_amd as rt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
W, H, S = 1200, 800, 500
r = rt.Renderer(rt.random_scene(), 0)
r.set_accel("grid")
cam = rt.final_camera(W / H)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
st = torch.cuda.current_stream().cuda_stream
for k in range(K + 1):
    r.set_ordering("cost")  # forgets the map: the next render probes first
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.render_rows(cam, W, H, S, 50, 1984, 0, 1, H, out.data_ptr(), st)
    torch.cuda.synchronize()
    if k:
        print(f"one-shot {k}: {(time.perf_counter() - t0) * 1e3:.3f} ms wall", flush=True)
r.close()
