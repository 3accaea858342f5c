"""The script behind queue_flake*.txt (analysis only; it needs the queue kernel,
retired in round 6 — run it against a build of 1b6ce15's experimental library):
N renders of 300x200x64 through RT_KERNEL_QUEUE, every other one after a
fault-injected render of another layout (RTMI_QUEUE_FAULT_INJECT=1), printing
each failure's message (which watchdog: ring take / ring put / idle block).
usage: RTMI_LIBRARY=.../librtmi_experimental.so python queue_flake.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import a_dive_into_ray_tracing_amd as rt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
r = rt.Renderer(rt.random_scene(), 0)
r.set_accel("grid")
r.set_kernel("queue")
cam = rt.final_camera(1.5)
ref = None
fails = 0
for k in range(n):
    if k % 2:
        os.environ["RTMI_QUEUE_FAULT_INJECT"] = "1"
        try:
            r.render(cam, 64, 40, 6, 50, 1984)
        except rt.RTError:
            pass
        del os.environ["RTMI_QUEUE_FAULT_INJECT"]
    try:
        img = r.render(cam, 300, 200, 64, 50, 1984)
        if ref is None:
            ref = img
        elif not np.array_equal(img, ref):
            print(f"render {k}: image differs", flush=True)
    except rt.RTError as e:
        fails += 1
        print(f"render {k} (after injection: {bool(k % 2)}): {e}", flush=True)
print(f"{fails} of {n} clean renders failed", flush=True)
r.close()
