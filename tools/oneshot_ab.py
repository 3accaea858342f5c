"""One-shot render time (the cost probe included) of config 2 and of one
rank's 1/8 strip, for the probe settings in the environment (RTMI_PROBE_DEPTH,
RTMI_PROBE_SPP; analysis only): K renders each forgetting the cost map, and a
steady render (the previous render's map) for reference; prints one JSON
line of medians (HIP events around each render on its stream)."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import a_dive_into_ray_tracing_amd as rt  # noqa: E402
from a_dive_into_ray_tracing_amd import dist as rdist  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
W, H, S = 1200, 800, 500
r = rt.Renderer(rt.random_scene(), 0)
r.set_accel("grid")
cam = rt.final_camera(W / H)
s = torch.cuda.Stream()
out = {"probe_depth": os.environ.get("RTMI_PROBE_DEPTH", "0"), "probe_spp": os.environ.get("RTMI_PROBE_SPP", "0")}
for name, strip_of in (("frame", 1), ("strip8", 8)):
    row0, step, nrows = rdist.strip_rows(H, 0, strip_of)
    buf = torch.empty((nrows, W, 3), dtype=torch.float32, device="cuda:0")

    def once():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r.render_rows(cam, W, H, S, 50, 1984, row0, step, nrows, buf.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    one, steady = [], []
    once()  # warm-up
    for _ in range(K):
        r.set_ordering("cost")  # forgets the map: the next render probes first
        one.append(once())
        steady.append(once())
    out[name] = {"one_shot_ms": round(statistics.median(one), 3), "steady_ms": round(statistics.median(steady), 3)}
print(json.dumps(out), flush=True)
r.close()
