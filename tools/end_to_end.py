"""End-to-end rates of config 2 beside bench.py's device-resident figure
(SURVEY §8(d) "also report end-to-end"):
  1. rt_render through the Python binding: the drop-in surface, which returns
     the sums in host memory (kernel + 11.5 MB device-to-host copy), steady
     (the context's cost map warm) and one-shot (a fresh context: cost probe);
  2. the C++ driver bin/rtmi_render as a process: HIP start-up, scene
     generation, render, P3 PPM written to a file (the reference's main()).
Prints one JSON line."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401  (one HIP runtime for the process)

import a_dive_into_ray_tracing_amd as rt  # noqa: E402

W, H, S, D, SEED = 1200, 800, 500, 50, 1984
samples = W * H * S
world = rt.random_scene()
cam = rt.final_camera(W / H)
out = {}

r = rt.Renderer(world, 0)
t0 = time.perf_counter()
r.render(cam, W, H, S, D, SEED)
out["rt_render_one_shot_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    r.render(cam, W, H, S, D, SEED)
    ts.append(time.perf_counter() - t0)
r.close()
out["rt_render_steady_ms"] = round(min(ts) * 1e3, 3)
out["rt_render_steady_msamples_per_s"] = round(samples / min(ts) / 1e6, 1)
out["rt_render_one_shot_msamples_per_s"] = round(samples / (out["rt_render_one_shot_ms"] * 1e-3) / 1e6, 1)

cli = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "bin", "rtmi_render")
ppm = os.path.join(REPO, "gpurun_out", "e2e_final.ppm")
os.makedirs(os.path.dirname(ppm), exist_ok=True)
walls = []
for _ in range(2):
    t0 = time.perf_counter()
    subprocess.run([cli, "--scene", "final", "--width", str(W), "--height", str(H), "--spp", str(S), "--depth", str(D),
                    "--seed", str(SEED), "--out", ppm], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    walls.append(time.perf_counter() - t0)
out["cli_process_wall_s"] = [round(w, 3) for w in walls]
out["cli_process_msamples_per_s"] = round(samples / min(walls) / 1e6, 1)
out["ppm_bytes"] = os.path.getsize(ppm)
os.remove(ppm)
print(json.dumps(out), flush=True)
