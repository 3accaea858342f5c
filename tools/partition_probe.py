"""Partition probe (analysis only): time each rank's share of an N-GPU render of
config 2 on ONE GPU, for interleaved rows (the production partition) and for
contiguous bands, to separate the strip's coherence cost from its dispatch tail.

    python tools/partition_probe.py [N] [tile_w] [bvh|none]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
import a_dive_into_ray_tracing_amd as rt  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
TW = int(sys.argv[2]) if len(sys.argv) > 2 else 8
W, H, SPP, DEPTH, SEED = 1200, 800, 500, 50, 1984
world = rt.random_scene()
cam = rt.final_camera(W / H)
r = rt.Renderer(world, 0, tile_w=TW)
r.set_accel(sys.argv[3] if len(sys.argv) > 3 else "bvh")
r.set_ordering("cost")
stream = torch.cuda.Stream(0)
torch.cuda.set_stream(stream)


def t_rows(row0, step, nrows, reps=3):
    out = torch.empty((nrows, W, 3), dtype=torch.float32, device="cuda:0")
    for _ in range(2):  # warmup (also primes the cost order of this layout)
        r.render_rows(cam, W, H, SPP, DEPTH, SEED, row0, step, nrows, out.data_ptr(), stream.cuda_stream)
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render_rows(cam, W, H, SPP, DEPTH, SEED, row0, step, nrows, out.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return min(ms)


full = t_rows(0, 1, H)
rows = H // N
inter = [t_rows(k, N, rows) for k in range(N)]
band = [t_rows(k * rows, 1, rows) for k in range(N)]
print(json.dumps({"N": N, "tile_w": TW, "full_ms": round(full, 3), "ideal_ms": round(full / N, 3),
                  "interleaved_ms": [round(x, 3) for x in inter], "interleaved_max": round(max(inter), 3),
                  "interleaved_sum": round(sum(inter), 3),
                  "band_ms": [round(x, 3) for x in band], "band_max": round(max(band), 3),
                  "band_sum": round(sum(band), 3)}))
