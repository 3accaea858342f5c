"""Analysis: render the Next-Week final scene (800x800) on the GPU and compare
it with the reference's gallery/final_scene_5000.png; writes our PNG, a
difference map and tile statistics under gpurun_out/nw/.  Not a test."""
import os
import sys
import time

import numpy as np
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402

OUT = os.path.join(REPO, "gpurun_out", "nw")
os.makedirs(OUT, exist_ok=True)
GOLD = os.path.join(REPO, "tests", "golden")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
earth = nw.load_image(os.path.join(GOLD, "earthmap.jpeg"))
ref = np.asarray(Image.open(os.path.join(GOLD, "gallery_final_scene_5000.png")).convert("RGB"), np.float64)
for tag, rtl in (("ltr", False), ("rtl", True)):
    s, cam = nw.preset("final", image=earth, aspect=1.0, rtl=rtl)
    r = nw.NwRenderer(s)
    r.render(cam, 64, 64, 1)
    t0 = time.time()
    img = r.render(cam, 800, 800, spp, 50, 1984)
    dt = time.time() - t0
    segs = r.last_segments()
    r.close()
    q = np.clip(np.floor(255.99 * np.sqrt(np.clip(img / spp, 0, None))), 0, 255)[::-1]
    Image.fromarray(q.astype(np.uint8)).save(os.path.join(OUT, f"final_{tag}_{spp}.png"))
    d = q - ref
    Image.fromarray(np.clip(128 + 2 * d.mean(axis=2), 0, 255).astype(np.uint8)).save(os.path.join(OUT, f"diff_{tag}_{spp}.png"))
    to = q.reshape(16, 50, 16, 50, 3).mean(axis=(1, 3))
    tr = ref.reshape(16, 50, 16, 50, 3).mean(axis=(1, 3))
    print(f"{tag}: {dt:.2f} s {800 * 800 * spp / dt / 1e6:.0f} Msamples/s seg/sample {segs / (800 * 800 * spp):.3f} "
          f"bias {d.mean():.2f} MAE {np.abs(d).mean():.2f} tile MAE {np.abs(to - tr).mean():.2f}", flush=True)
    np.save(os.path.join(OUT, f"tiles_{tag}.npy"), to - tr)
