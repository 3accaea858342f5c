"""Brute-force vs BVH closest hit on many random rays (GPU box); prints the
mismatches.  usage: python tools/bvh_hits.py [n_rays]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import a_dive_into_ray_tracing_amd as rt  # noqa: E402

L = rt.load()
L.rt_ctx_debug_hits.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_float)]
w = rt.random_scene()
r = rt.Renderer(w, 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
g = np.random.default_rng(5)
o = np.column_stack([g.uniform(-13, 13, n), g.uniform(-0.1, 3, n), g.uniform(-13, 13, n)])
# half the origins just off sphere surfaces (bounce origins)
k = g.integers(0, len(w), n // 2)
c, rad = w.center_radius[k, :3], np.abs(w.center_radius[k, 3])
u = g.normal(size=(n // 2, 3))
u /= np.linalg.norm(u, axis=1, keepdims=True)
o[: n // 2] = c + u * (rad[:, None] * (1 + g.choice([1e-3, 1e-4, -1e-4, 1e-6], n // 2)[:, None]))
dvec = g.normal(size=(n, 3)) * g.choice([0.3, 1.0, 3.0], n)[:, None]
zero = g.random((n, 3)) < 0.02  # some exactly-zero components
dvec[zero] = 0.0
dvec[np.all(dvec == 0, axis=1)] = [0, -1, 0]
rays = np.ascontiguousarray(np.column_stack([o, dvec]).astype(np.float32))
idx = np.zeros(2 * n, np.int32)
t = np.zeros(2 * n, np.float32)
rc = L.rt_ctx_debug_hits(r._h, rays.ctypes.data_as(C.POINTER(C.c_float)), n, idx.ctypes.data_as(C.POINTER(C.c_int32)),
                         t.ctypes.data_as(C.POINTER(C.c_float)))
assert rc == 0, L.rt_last_error()
idx = idx.reshape(n, 2)
t = t.reshape(n, 2)
bad = np.where((idx[:, 0] != idx[:, 1]) | ((t[:, 0] != t[:, 1]) & (idx[:, 0] >= 0)))[0]
print(f"rays {n}: hits {np.mean(idx[:, 0] >= 0):.3f}, mismatches {len(bad)}")
for b in bad[:20]:
    print(f"  ray {b}: o {rays[b, :3]} d {rays[b, 3:]} brute ({idx[b, 0]}, {t[b, 0]!r}) bvh ({idx[b, 1]}, {t[b, 1]!r})")
