"""tests/oracle_py.py — ctypes view of oracle/build/liboracle.so (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It is the checker: nothing in the product path calls it.
"""
import ctypes as C
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("ORACLE_LIBRARY") or os.path.join(REPO, "oracle", "build", "liboracle.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int32)
_lp = C.POINTER(C.c_int64)


class OrScene(C.Structure):
    _fields_ = [("n", C.c_int32), ("geom", _dp), ("kind", _ip), ("mat", _dp)]


class OrCamera(C.Structure):
    _fields_ = [(nm, C.c_double * 3) for nm in ("origin", "lower_left_corner", "horizontal", "vertical", "u", "v", "w")] + [
        ("lens_radius", C.c_double)
    ]


class OrGlibc(C.Structure):
    _fields_ = [("state", C.c_int32 * 31), ("f", C.c_int32), ("r", C.c_int32), ("draws", C.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(LIB_PATH)
        L.or_glibc_seed.argtypes = [C.POINTER(OrGlibc), C.c_uint32]
        L.or_glibc_rand.argtypes = [C.POINTER(OrGlibc)]
        L.or_glibc_rand.restype = C.c_int32
        L.or_final_scene.argtypes = [C.POINTER(OrGlibc), _dp, _ip, _dp, C.c_int32]
        L.or_final_scene.restype = C.c_int32
        L.or_learn_scene.argtypes = [_dp, _ip, _dp, C.c_int32]
        L.or_learn_scene.restype = C.c_int32
        L.or_camera_make.argtypes = [C.POINTER(OrCamera), _dp, _dp, _dp, C.c_double, C.c_double, C.c_double, C.c_double]
        L.or_ref_worker.argtypes = [C.POINTER(OrScene), C.POINTER(OrCamera)] + [C.c_int32] * 6 + [C.POINTER(OrGlibc), _dp]
        L.or_ref_worker.restype = C.c_int64
        L.or_ref_last_segments.restype = C.c_int64
        L.or_ref_kat.argtypes = [C.POINTER(OrScene), C.POINTER(OrCamera)] + [C.c_int32] * 5 + [C.c_uint32, _dp]
        L.or_ref_kat.restype = C.c_int32
        L.or_ref_sphere_hit.argtypes = [_dp, C.c_double, _dp, _dp, C.c_double, C.c_double, _dp, _dp, _dp, _ip]
        L.or_ref_sphere_hit.restype = C.c_int32
        L.or_ref_refract.argtypes = [_dp, _dp, C.c_double, _dp]
        L.or_ref_reflect.argtypes = [_dp, _dp, _dp]
        L.or_ref_reflectance.argtypes = [C.c_double, C.c_double]
        L.or_ref_reflectance.restype = C.c_double
        L.or_ref_near_zero.argtypes = [_dp]
        L.or_ref_near_zero.restype = C.c_int32
        L.or_ref_scatter.argtypes = [C.c_int32, _dp, _dp, _dp, _dp, C.c_int32, C.c_uint32, _dp, _dp, _dp, _ip]
        L.or_ref_scatter.restype = C.c_int32
        fast_args = [C.POINTER(OrScene), C.POINTER(OrCamera)] + [C.c_int32] * 4 + [C.c_uint64] + [C.c_int32] * 3
        L.or_fast_render.argtypes = fast_args + [_fp]
        L.or_fast_render.restype = C.c_int32
        L.or_fast_render_fixed.argtypes = fast_args + [_lp]
        L.or_fast_render_fixed.restype = C.c_int32
        L.or_fast_segments.argtypes = fast_args
        L.or_fast_segments.restype = C.c_int64
        L.or_fast_sample.argtypes = [C.POINTER(OrScene), C.POINTER(OrCamera)] + [C.c_int32] * 3 + [C.c_uint64] + [C.c_int32] * 3 + [_fp]
        L.or_fast_sample.restype = C.c_int32
        L.or_fast_rng.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_int32, C.POINTER(C.c_uint64)]
        L.or_fast_dirs.argtypes = [C.c_int32, C.c_uint64, C.c_int32, C.POINTER(C.c_float)]
        _lib = L
    return _lib


def dptr(a):
    return a.ctypes.data_as(_dp)


class Scene:
    """Flat scene arrays (geom 4n, kind n, mat 4n) + the ctypes struct."""

    def __init__(self, geom, kind, mat):
        self.geom = np.ascontiguousarray(geom, dtype=np.float64).reshape(-1)
        self.kind = np.ascontiguousarray(kind, dtype=np.int32).reshape(-1)
        self.mat = np.ascontiguousarray(mat, dtype=np.float64).reshape(-1)
        self.n = self.kind.size
        self.c = OrScene(self.n, dptr(self.geom), self.kind.ctypes.data_as(_ip), dptr(self.mat))


def final_scene():
    """random_scene() from the seed-1 stream; returns (Scene, stream after it)."""
    g = OrGlibc()
    lib().or_glibc_seed(C.byref(g), 1)
    geom = np.zeros(4 * 600)
    kind = np.zeros(600, np.int32)
    mat = np.zeros(4 * 600)
    n = lib().or_final_scene(C.byref(g), dptr(geom), kind.ctypes.data_as(_ip), dptr(mat), 600)
    return Scene(geom[: 4 * n], kind[:n], mat[: 4 * n]), g


def learn_scene():
    geom = np.zeros(20)
    kind = np.zeros(5, np.int32)
    mat = np.zeros(20)
    lib().or_learn_scene(dptr(geom), kind.ctypes.data_as(_ip), dptr(mat), 5)
    return Scene(geom, kind, mat)


def make_camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus):
    c = OrCamera()
    a = [np.asarray(x, dtype=np.float64) for x in (lookfrom, lookat, vup)]
    lib().or_camera_make(C.byref(c), dptr(a[0]), dptr(a[1]), dptr(a[2]), vfov, aspect, aperture, focus)
    return c


def final_camera(aspect=1.5):
    return make_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, aspect, 0.1, 10.0)


def learn_camera(aspect=16.0 / 9.0):
    lf, la = np.array([3.0, 3, 2]), np.array([0.0, 0, -1])
    d = lf - la
    focus = float(np.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]))
    return make_camera(lf, la, (0, 1, 0), 20.0, aspect, 0.5, focus)


def camera_dict(c):
    return {nm: list(getattr(c, nm)) for nm in ("origin", "lower_left_corner", "horizontal", "vertical", "u", "v", "w")} | {
        "lens_radius": c.lens_radius
    }


def ref_worker(scene, cam, W, H, spp, depth, start, end, g):
    out = np.zeros((end - start) * 3)
    draws = lib().or_ref_worker(C.byref(scene.c), C.byref(cam), W, H, spp, depth, start, end, C.byref(g), dptr(out))
    return out, draws


def ref_kat(scene, cam, W, H, depth, i, j, seed):
    out = np.zeros(3)
    nxt = lib().or_ref_kat(C.byref(scene.c), C.byref(cam), W, H, depth, i, j, seed, dptr(out))
    return out, nxt


def fast_render(scene, cam, W, H, spp, depth, seed, row0=0, row_step=1, nrows=None, fixed=False):
    nrows = H if nrows is None else nrows
    if fixed:
        out = np.zeros(nrows * W * 3, np.int64)
        rc = lib().or_fast_render_fixed(C.byref(scene.c), C.byref(cam), W, H, spp, depth, seed, row0, row_step, nrows, out.ctypes.data_as(_lp))
    else:
        out = np.zeros(nrows * W * 3, np.float32)
        rc = lib().or_fast_render(C.byref(scene.c), C.byref(cam), W, H, spp, depth, seed, row0, row_step, nrows, out.ctypes.data_as(_fp))
    if rc != 0:
        raise ValueError("or_fast_render failed")
    return out.reshape(nrows, W, 3)


def fast_segments(scene, cam, W, H, spp, depth, seed, row0=0, row_step=1, nrows=None):
    nrows = H if nrows is None else nrows
    return lib().or_fast_segments(C.byref(scene.c), C.byref(cam), W, H, spp, depth, seed, row0, row_step, nrows)


def load_scene_txt(path):
    rows = open(path).read().split("\n")
    n = int(rows[0])
    data = [r.split() for r in rows[1 : 1 + n]]
    geom = np.array([[float(x) for x in r[:4]] for r in data])
    kind = np.array([int(r[4]) for r in data], np.int32)
    mat = np.array([[float(x) for x in r[5:9]] for r in data])
    return Scene(geom, kind, mat)


def load_camera_txt(path):
    out = {}
    for line in open(path):
        t = line.split()
        vals = [float(x) for x in t[1:]]
        out[t[0]] = vals if len(vals) > 1 else vals[0]
    return out


# ---- Next-Week restatement (oracle/rt_nw_oracle.inc) ----------------------
class OrNwScene(C.Structure):
    _fields_ = [("n_obj", C.c_int32), ("n_inst", C.c_int32)] + [
        (nm, _fp) for nm in ("obj", "inst", "mat", "tex", "perlin_vec")
    ] + [("perlin_perm", _ip), ("image_desc", _ip), ("image_px", C.POINTER(C.c_uint8)), ("bg", C.c_float * 3)]


def _nw_bind():
    L = lib()
    if not getattr(L, "_nw_bound", False):
        L.or_nw_render.argtypes = [C.POINTER(OrNwScene), C.POINTER(OrCamera), C.c_double, C.c_double] + [C.c_int32] * 4 + [
            C.c_uint64] + [C.c_int32] * 3 + [_fp, _lp]
        L.or_nw_render.restype = C.c_int32
        L.or_nw_math.argtypes = [C.c_int32, C.c_int32, _fp, _fp]
        L._nw_bound = True
    return L


def nw_scene(flat):
    """OrNwScene over the arrays of nextweek.Scene.flat() (kept alive on the struct)."""
    keep = {k: (np.ascontiguousarray(v) if isinstance(v, np.ndarray) else v) for k, v in flat.items()}
    for k in ("obj", "inst", "mat", "tex", "perlin_vec", "perlin_perm", "image_desc", "image_px"):
        if keep[k].size == 0:
            keep[k] = np.zeros(16, keep[k].dtype)
    s = OrNwScene()
    s.n_obj = int(flat["n_obj"])
    s.n_inst = int(flat["inst"].size // 8)
    for k in ("obj", "inst", "mat", "tex", "perlin_vec"):
        setattr(s, k, keep[k].ctypes.data_as(_fp))
    s.perlin_perm = keep["perlin_perm"].ctypes.data_as(_ip)
    s.image_desc = keep["image_desc"].ctypes.data_as(_ip)
    s.image_px = keep["image_px"].ctypes.data_as(C.POINTER(C.c_uint8))
    for c in range(3):
        s.bg[c] = float(flat["background"][c])
    s._keep = keep
    return s


def nw_render(flat, nwcam, W, H, spp, depth, seed, row0=0, row_step=1, nrows=None):
    """Oracle image (sums) + world.hit count for rows row0 + r*row_step of a W x H Next-Week render."""
    L = _nw_bind()
    nrows = H if nrows is None else nrows
    s = nw_scene(flat)
    cam = OrCamera()
    C.memmove(C.byref(cam), C.byref(nwcam.cam), C.sizeof(cam))
    out = np.zeros(nrows * W * 3, np.float32)
    segs = C.c_int64()
    rc = L.or_nw_render(C.byref(s), C.byref(cam), nwcam.time0, nwcam.time1, W, H, spp, depth, seed, row0, row_step,
                        nrows, out.ctypes.data_as(_fp), C.byref(segs))
    if rc != 0:
        raise ValueError("or_nw_render failed")
    return out.reshape(nrows, W, 3), segs.value


def nw_math(fn, x):
    L = _nw_bind()
    x = np.ascontiguousarray(x, np.float32)
    n = x.size // 2 if fn == 2 else x.size
    out = np.zeros(n, np.float32)
    L.or_nw_math(fn, n, x.ctypes.data_as(_fp), out.ctypes.data_as(_fp))
    return out


def nw_box_forms(rays, boxes):
    """or_nw_box_forms: (t, face) of each ray against its box, division form
    and reciprocal form."""
    L = _nw_bind()
    L.or_nw_box_forms.argtypes = [C.c_int32, _fp, _fp, _fp, _ip, _fp, _ip]
    rays = np.ascontiguousarray(rays, np.float32)
    boxes = np.ascontiguousarray(boxes, np.float32)
    n = rays.shape[0]
    td, ti = np.zeros(n, np.float32), np.zeros(n, np.float32)
    fd, fi = np.zeros(n, np.int32), np.zeros(n, np.int32)
    L.or_nw_box_forms(n, rays.ctypes.data_as(_fp), boxes.ctypes.data_as(_fp), td.ctypes.data_as(_fp),
                      fd.ctypes.data_as(_ip), ti.ctypes.data_as(_fp), fi.ctypes.data_as(_ip))
    return td, fd, ti, fi


def nw_trace(flat, nwcam, W, H, depth, seed, i, j, smp, cap=64):
    """Oracle mirror of NwRenderer.debug_trace."""
    L = _nw_bind()
    L.or_nw_trace.argtypes = [C.POINTER(OrNwScene), C.POINTER(OrCamera), C.c_double, C.c_double] + [C.c_int32] * 3 + [
        C.c_uint64] + [C.c_int32] * 3 + [_fp, C.c_int32]
    L.or_nw_trace.restype = C.c_int32
    s = nw_scene(flat)
    cam = OrCamera()
    C.memmove(C.byref(cam), C.byref(nwcam.cam), C.sizeof(cam))
    rec = np.zeros(12 * cap, np.float32)
    n = L.or_nw_trace(C.byref(s), C.byref(cam), nwcam.time0, nwcam.time1, W, H, depth, seed, i, j, smp,
                      rec.ctypes.data_as(_fp), cap)
    out = rec[: 12 * n].reshape(-1, 12).copy()
    return out[:, [0, 1, 2, 3, 4, 5, 6, 8, 9, 10]], out[:, [7, 11]].view(np.int32)


def nw_hits(flat, rays, keys=None):
    """Oracle mirror of NwRenderer.debug_hits: the brute-force closest hit of
    each ray (rows o.xyz, d.xyz, time): (insertion index or -1, t, box face)."""
    L = _nw_bind()
    L.or_nw_hits.argtypes = [C.POINTER(OrNwScene), _fp, C.POINTER(C.c_uint64), C.c_int32, _ip, _fp, _ip]
    L.or_nw_hits.restype = None
    s = nw_scene(flat)
    n = len(rays)
    r = np.zeros((n, 8), np.float32)
    r[:, :7] = rays
    k = None if keys is None else np.ascontiguousarray(keys, np.uint64)
    idx, t, face = np.zeros(n, np.int32), np.zeros(n, np.float32), np.zeros(n, np.int32)
    L.or_nw_hits(C.byref(s), r.ctypes.data_as(_fp), None if k is None else k.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                 idx.ctypes.data_as(_ip), t.ctypes.data_as(_fp), face.ctypes.data_as(_ip))
    return idx, t, face


def row_mean_z(frame_rows, S, a, b, s_ab):
    """Per-row, per-channel z-scores of a frame's row means against two
    independent oracle renders of the same rows (sums at s_ab spp under two
    other seeds), and the mean of z^2 (chi-square per degree of freedom).
    The noise of a row mean is measured, not assumed: the per-pixel
    difference of the two oracle renders has variance 2 s^2 / s_ab per pixel
    (s^2 the per-sample variance), pooled over the row's pixels; the frame's
    own noise (S spp) is added at the same per-sample variance."""
    f = np.asarray(frame_rows, np.float64) / S
    ma, mb = np.asarray(a, np.float64) / s_ab, np.asarray(b, np.float64) / s_ab
    W = f.shape[1]
    var1 = s_ab * ((ma - mb) ** 2).mean(axis=1) / 2.0  # per-sample variance, per row and channel
    var_ref = var1 / (2 * s_ab * W)  # the mean of the two oracle renders' row means
    var_frame = var1 / (S * W)
    d = f.mean(axis=1) - (ma + mb).mean(axis=1) / 2.0
    z = d / np.sqrt(var_ref + var_frame + 1e-30)
    return z, float((z ** 2).mean())
