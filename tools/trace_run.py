"""Per-wave timeline of the RTMI_TRACE build (run on the GPU box).

usage: python tools/trace_run.py [grid|persistent] [strip_of] [chunk] [tail_spp] [tail_chunk]
Prints the kernel span, the wave-end percentiles and how many waves are
resident over time (10 bins), i.e. where the dispatch tail is.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["RTMI_LIBRARY"] = os.path.join(ROOT, "a_dive_into_ray_tracing_amd", "lib", os.environ.get("TRACE_LIB", "librtmi_trace.so"))
import torch  # noqa: E402,F401  (one HIP runtime)
import a_dive_into_ray_tracing_amd as rt  # noqa: E402
from a_dive_into_ray_tracing_amd import dist as rdist  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "persistent"
strip_of = int(sys.argv[2]) if len(sys.argv) > 2 else 1
chunk, tail, tchunk = (int(x) for x in (sys.argv[3:6] + ["0", "-1", "0"][len(sys.argv[3:6]):]))
L = rt.load()
L.rt_ctx_debug_trace.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
L.rt_ctx_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
W, H, S = 1200, 800, 500
r = rt.Renderer(rt.random_scene(), 0)
r.set_kernel(kind)
r.set_accel(os.environ.get("TRACE_ACCEL", "none"))
r.set_schedule(chunk, tail, tchunk)
cam = rt.final_camera(1.5)
row0, step, nrows = rdist.strip_rows(H, 0, strip_of)
strip = torch.empty((nrows, W, 3), dtype=torch.float32, device="cuda:0")
cap = 1 << 18
buf = (C.c_uint64 * (4 * cap))()
for it in range(2):
    r.render_rows(cam, W, H, S, 50, 1984, row0, step, nrows, strip.data_ptr(), 0)
    r.synchronize()
    cnt = (C.c_uint64 * 8)()
    L.rt_ctx_debug_counters(r._h, cnt)
    n = L.rt_ctx_debug_trace(r._h, buf, cap)
t = np.frombuffer(buf, dtype=np.uint64, count=4 * n).reshape(n, 4).astype(np.float64)
t0, t1 = t[:, 0], t[:, 1]
base = t0.min()
t0 = (t0 - base) / 100.0  # us (100 MHz)
t1 = (t1 - base) / 100.0
span = t1.max()
items = (t[:, 2].astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.int64)
raw = np.frombuffer(buf, dtype=np.uint64, count=4 * n).reshape(n, 4)
segs = (raw[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.float64)
wid = (raw[:, 3] >> np.uint64(32)).astype(np.int64)
hw = (raw[:, 2] >> np.uint64(32)).astype(np.int64)
print(f"{kind} strip_of={strip_of} chunk={chunk} tail={tail}/{tchunk}: waves {n}, span {span / 1e3:.2f} ms, "
      f"items {items.sum()}, segs/wave-line mean {segs.mean():.0f}")
print(f"cycles in hit_world_packed / wave lifetime: {cnt[5] / max(cnt[6], 1):.3f}")
if os.environ.get("TRACE_PHASES"):
    print(f"grid phases / wave lifetime: big spheres + clip/setup {cnt[1] / max(cnt[6], 1):.3f}, ramp-down passes {cnt[2] / max(cnt[6], 1):.3f}, cell walk {cnt[3] / max(cnt[6], 1):.3f}")
    print(f"loop passes / wave lifetime: hit + shading {cnt[4] / max(cnt[6], 1):.3f}, accumulation + regeneration {cnt[7] / max(cnt[6], 1):.3f}")
print("wave end percentiles (ms):", " ".join(f"p{q}={np.percentile(t1, q) / 1e3:.2f}" for q in (1, 10, 50, 90, 99, 100)))
print("wave duration percentiles (ms):", " ".join(f"p{q}={np.percentile(t1 - t0, q) / 1e3:.3f}" for q in (1, 10, 50, 90, 99, 100)))
bins = np.linspace(0, span, 21)
mid = 0.5 * (bins[1:] + bins[:-1])
res = [int(((t0 <= m) & (t1 > m)).sum()) for m in mid]
print("resident waves over time (20 bins):", res)
order = np.argsort(t1)[::-1][:12]
# HW_ID (gfx9 layout): wave_id [3:0], simd_id [5:4], cu_id [11:8], sh_id [12], se_id [15:13]
slot, simd, cu, se = hw & 15, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
print("latest waves: end_ms items segs wave# se cu simd slot")
for k in order:
    print(f"  {t1[k] / 1e3:8.2f} {items[k]:6d} {segs[k]:10.0f} {wid[k]:6d} {se[k]} {cu[k]:2d} {simd[k]} {slot[k]:2d}")
if kind == "persistent":
    # work per wave against its launch order among the waves of its SIMD
    key = se * 64 + cu * 4 + simd
    rank = np.zeros(n, np.int64)
    for kk in np.unique(key):
        idx = np.where(key == kk)[0]
        rank[idx[np.argsort(wid[idx])]] = np.arange(len(idx))
    for rr in range(int(rank.max()) + 1):
        sel = rank == rr
        print(f"  launch rank {rr} on its SIMD: waves {sel.sum():5d} mean segs {segs[sel].mean():9.0f}")
    for s_ in range(int(slot.max()) + 1):
        sel = slot == s_
        if sel.any():
            print(f"  hw slot {s_}: waves {sel.sum():5d} mean segs {segs[sel].mean():9.0f}")
print(f"segs per wave: p1 {np.percentile(segs, 1):.0f} p50 {np.percentile(segs, 50):.0f} p99 {np.percentile(segs, 99):.0f} max {segs.max():.0f}")
