"""a_dive_into_ray_tracing_amd — MI355X-native path tracer for the RTIOW final scene.

Python view of librtmi.so (include/rtmi.h), used by the tests and bench.py.
The product is the C ABI and its HIP kernels; this module only marshals
arrays.  Names mirror the reference (rt_in_one_weekend/):

    world = random_scene()                      # main.cpp:86-131
    cam = camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus)  # camera.h:8-45
    sums = render(W, H, spp, max_depth, world, cam)   # worker() main.cpp:267-290
    write_ppm("-", sums, spp)                   # write_color color.h:14-28

There is no CPU fallback: render() raises RTError(RT_ENODEVICE) without a
gfx950 GPU.
"""
import ctypes as C

import numpy as np

from . import _abi
from ._abi import RT_MAT_DIELECTRIC, RT_MAT_LAMBERTIAN, RT_MAT_METAL, RtCamera, RTError, RtScene, check, load

__all__ = [
    "RTError", "World", "lambertian", "metal", "dielectric", "sphere", "random_scene", "learn_scene",
    "camera", "final_camera", "learn_camera", "Renderer", "render", "quantize", "write_ppm", "device_count",
    "write_pfm", "read_pfm", "load_scene",
]

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int32)


def _d(a):
    return a.ctypes.data_as(_dp)


# ---------------------------------------------------------------- scene ----
def lambertian(albedo):
    """material.h:15-35"""
    return (RT_MAT_LAMBERTIAN, (float(albedo[0]), float(albedo[1]), float(albedo[2]), 0.0))


def metal(albedo, fuzz):
    """material.h:37-54 (fuzz clamped to 1 as the constructor does, :39)"""
    f = float(fuzz)
    return (RT_MAT_METAL, (float(albedo[0]), float(albedo[1]), float(albedo[2]), f if f < 1 else 1.0))


def dielectric(ir):
    """material.h:56-97"""
    return (RT_MAT_DIELECTRIC, (0.0, 0.0, 0.0, float(ir)))


def sphere(center, radius, material):
    """sphere.h:7-19"""
    return (tuple(float(c) for c in center), float(radius), material)


class World:
    """hittable_list of spheres (hittable_list.h:6-18) as the flat arrays of rt_scene."""

    def __init__(self, center_radius=None, mat_kind=None, mat_params=None):
        self.center_radius = np.zeros((0, 4)) if center_radius is None else np.asarray(center_radius, np.float64).reshape(-1, 4)
        self.mat_kind = np.zeros(0, np.int32) if mat_kind is None else np.asarray(mat_kind, np.int32).reshape(-1)
        self.mat_params = np.zeros((0, 4)) if mat_params is None else np.asarray(mat_params, np.float64).reshape(-1, 4)

    def add(self, obj):
        (center, radius, (kind, params)) = obj
        self.center_radius = np.vstack([self.center_radius, [*center, radius]])
        self.mat_kind = np.append(self.mat_kind, np.int32(kind))
        self.mat_params = np.vstack([self.mat_params, params])
        return self

    def __len__(self):
        return int(self.mat_kind.size)

    def save(self, path):
        """Scene text file (rt_scene_write; the format of tests/golden/scene_final.txt)."""
        sc = self.c_struct()
        check(load().rt_scene_write(str(path).encode(), C.byref(sc)), "rt_scene_write")

    def digest(self):
        """sha256 of the scene arrays (checkpoint headers)."""
        import hashlib

        h = hashlib.sha256()
        for a in (self.center_radius, self.mat_kind, self.mat_params):
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()

    def c_struct(self):
        self._keep = [np.ascontiguousarray(self.center_radius), np.ascontiguousarray(self.mat_kind), np.ascontiguousarray(self.mat_params)]
        g, k, m = self._keep
        return RtScene(len(self), _d(g), k.ctypes.data_as(_ip), _d(m))


def random_scene(glibc_seed=1):
    """random_scene() main.cpp:86-131 (487 spheres for the reference's seed 1)."""
    L = load()
    g, m = np.zeros(4 * 1024), np.zeros(4 * 1024)
    k = np.zeros(1024, np.int32)
    n = C.c_int32()
    check(L.rt_scene_random(glibc_seed, _d(g), k.ctypes.data_as(_ip), _d(m), 1024, C.byref(n)), "rt_scene_random")
    return World(g[: 4 * n.value], k[: n.value], m[: 4 * n.value])


def load_scene(path):
    """Scene text file -> World (rt_scene_read)."""
    L = load()
    n = C.c_int32()
    rc = L.rt_scene_read(str(path).encode(), None, None, None, 0, C.byref(n))
    if rc != 0 and n.value == 0:
        check(rc, "rt_scene_read")
    g, m = np.zeros(4 * max(n.value, 1)), np.zeros(4 * max(n.value, 1))
    k = np.zeros(max(n.value, 1), np.int32)
    check(L.rt_scene_read(str(path).encode(), _d(g), k.ctypes.data_as(_ip), _d(m), n.value, C.byref(n)), "rt_scene_read")
    return World(g[: 4 * n.value], k[: n.value], m[: 4 * n.value])


def learn_scene():
    """learn() world main.cpp:198-210 (config 1)."""
    L = load()
    g, m = np.zeros(20), np.zeros(20)
    k = np.zeros(5, np.int32)
    n = C.c_int32()
    check(L.rt_scene_learn(_d(g), k.ctypes.data_as(_ip), _d(m), 5, C.byref(n)), "rt_scene_learn")
    return World(g, k, m)


# --------------------------------------------------------------- camera ----
def camera(lookfrom, lookat, vup, vfov, aspect_ratio, aperture, focus_dist):
    """camera::camera camera.h:8-45 -> RtCamera (public fields camera.h:64-70)."""
    cam = RtCamera()
    a = [np.ascontiguousarray(x, dtype=np.float64) for x in (lookfrom, lookat, vup)]
    check(load().rt_camera_init(C.byref(cam), _d(a[0]), _d(a[1]), _d(a[2]), vfov, aspect_ratio, aperture, focus_dist), "rt_camera_init")
    return cam


def final_camera(aspect_ratio=1.5):
    """parallel_render() camera main.cpp:304-311"""
    return camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, aspect_ratio, 0.1, 10.0)


def learn_camera(aspect_ratio=16.0 / 9.0):
    """learn() camera main.cpp:212-221"""
    lf, la = np.array([3.0, 3.0, 2.0]), np.array([0.0, 0.0, -1.0])
    d = lf - la
    return camera(lf, la, (0, 1, 0), 20.0, aspect_ratio, 0.5, float(np.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])))


# ---------------------------------------------------------------- render ---
def device_count():
    n = C.c_int32(0)
    rc = load().rt_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def auto_tile_w(W, rows):
    """The tile width `rt_render_rows` picks when tile_w is 0 (rtmi_device.hip
    auto_tile_w): 8 unless 16x4 tiles leave fewer idle lanes in partial tiles."""
    def idle(tw):
        th = 64 // tw
        return -(-W // tw) * tw * (-(-rows // th)) * th - W * rows
    return 16 if idle(16) < idle(8) else 8


class Renderer:
    """One rt_ctx: a device, its stream and the resident scene."""

    def __init__(self, world, device=0, tile_w=0, chunk=0):
        self.L = load()
        self._h = C.c_void_p()
        check(self.L.rt_ctx_create(device, C.byref(self._h)), "rt_ctx_create")
        self.device = device
        self.set_scene(world)
        self.set_tuning(tile_w, chunk)

    def set_scene(self, world):
        sc = world.c_struct()
        check(self.L.rt_ctx_set_scene(self._h, C.byref(sc)), "rt_ctx_set_scene")
        self.world = world

    def set_tuning(self, tile_w=0, chunk=0):
        check(self.L.rt_ctx_set_tuning(self._h, tile_w, chunk), "rt_ctx_set_tuning")

    def set_schedule(self, chunk=0, tail_spp=-1, tail_chunk=0):
        check(self.L.rt_ctx_set_schedule(self._h, chunk, tail_spp, tail_chunk), "rt_ctx_set_schedule")

    def set_overlap(self, overlapped=True):
        """Launch-mode hint: this context's renders overlap another context's on
        the same device (rt_ctx_set_overlap); fewer, longer work items."""
        check(self.L.rt_ctx_set_overlap(self._h, int(bool(overlapped))), "rt_ctx_set_overlap")

    KERNELS = {"grid": 0, "persistent": 1, "auto": 2, "queue": 3, "resident": 4}  # RT_KERNEL_* (include/rtmi.h)

    def set_kernel(self, kind="auto"):
        check(self.L.rt_ctx_set_kernel(self._h, self.KERNELS[kind]), "rt_ctx_set_kernel")

    ORDERINGS = {"none": 0, "cost": 1}  # RT_ORDER_* (include/rtmi.h)

    def set_ordering(self, ordering="cost"):
        check(self.L.rt_ctx_set_ordering(self._h, self.ORDERINGS[ordering]), "rt_ctx_set_ordering")

    ACCELS = {"none": 0, "bvh": 1, "grid": 2}  # RT_ACCEL_* (include/rtmi.h)

    def set_accel(self, accel="none"):
        check(self.L.rt_ctx_set_accel(self._h, self.ACCELS[accel]), "rt_ctx_set_accel")

    def accel_info(self):
        """(big spheres tested brute force, BVH nodes) for the current scene."""
        nb, nn = C.c_int32(), C.c_int32()
        check(self.L.rt_ctx_accel_info(self._h, C.byref(nb), C.byref(nn)), "rt_ctx_accel_info")
        return nb.value, nn.value

    def grid_info(self):
        """((nx, ny, nz) cells, references, LDS bytes) of the scene's uniform grid."""
        dims, nr, lds = (C.c_int32 * 3)(), C.c_int32(), C.c_int32()
        check(self.L.rt_ctx_grid_info(self._h, dims, C.byref(nr), C.byref(lds)), "rt_ctx_grid_info")
        return tuple(dims), nr.value, lds.value

    def render(self, cam, W, H, spp, max_depth=50, seed=1984):
        """Whole image, host float32 sums [H, W, 3], row 0 = bottom (main.cpp:274)."""
        out = np.zeros(W * H * 3, np.float32)
        check(self.L.rt_render(self._h, C.byref(cam), W, H, spp, max_depth, seed, out.ctypes.data_as(_fp)), "rt_render")
        return out.reshape(H, W, 3)

    def render_rows(self, cam, W, H, spp, max_depth, seed, row0, row_step, nrows, dev_ptr, stream=0):
        """Rows row0 + r*row_step into a device strip (async on `stream`)."""
        check(
            self.L.rt_render_rows(self._h, C.byref(cam), W, H, spp, max_depth, seed, row0, row_step, nrows, C.c_void_p(dev_ptr), C.c_void_p(stream)),
            "rt_render_rows",
        )

    def last_segments(self):
        """world.hit calls of the last render (GPU-counted)."""
        v = C.c_uint64()
        check(self.L.rt_ctx_last_segments(self._h, C.byref(v)), "rt_ctx_last_segments")
        return v.value

    def last_schedule(self):
        """Diagnostic: the last launch's schedule as a dict (rt_ctx_last_schedule)."""
        v = (C.c_int32 * 8)()
        check(self.L.rt_ctx_last_schedule(self._h, v), "rt_ctx_last_schedule")
        keys = ("tile_w", "chunk", "items_per_tile", "tail_items_per_tile", "block_flush", "ray_pool", "persistent", "bvh")
        return dict(zip(keys, list(v)))

    def synchronize(self):
        check(self.L.rt_ctx_synchronize(self._h), "rt_ctx_synchronize")

    def replay_worker(self, cam, W, H, spp, max_depth, jobs, streams):
        """Exact (double) replay of reference worker(start,end) calls with supplied rand() streams.
        jobs: [(start, end), ...]; streams: list of int32 arrays (one per job)."""
        ranges = np.ascontiguousarray(np.asarray(jobs, np.int32).reshape(-1))
        offs = np.zeros(len(jobs) + 1, np.int64)
        offs[1:] = np.cumsum([len(s) for s in streams])
        flat = np.ascontiguousarray(np.concatenate([np.asarray(s, np.int32) for s in streams]) if offs[-1] else np.zeros(1, np.int32))
        total = sum(3 * (e - s) for s, e in jobs)
        out = np.zeros(max(total, 1))
        used = np.zeros(len(jobs), np.int64)
        check(
            self.L.rt_replay_worker(
                self._h, C.byref(cam), W, H, spp, max_depth, len(jobs), ranges.ctypes.data_as(_ip), flat.ctypes.data_as(_ip),
                offs.ctypes.data_as(C.POINTER(C.c_int64)), _d(out), used.ctypes.data_as(C.POINTER(C.c_int64)),
            ),
            "rt_replay_worker",
        )
        return out[:total], used

    # ---- progressive accumulation (rt_accum_* / rt_render_pass) ----------
    def accum_reset(self, W, nrows):
        check(self.L.rt_accum_reset(self._h, W, nrows), "rt_accum_reset")
        self._acc_shape = (nrows, W, 3)

    def render_pass(self, cam, W, H, s_begin, s_count, max_depth=50, seed=1984, row0=0, row_step=1, nrows=None, stream=0):
        """Add samples [s_begin, s_begin + s_count) of the rows to the accumulator (async)."""
        nrows = H if nrows is None else nrows
        check(
            self.L.rt_render_pass(self._h, C.byref(cam), W, H, s_begin, s_count, max_depth, seed, row0, row_step, nrows, C.c_void_p(stream)),
            "rt_render_pass",
        )

    def accum_resolve(self):
        """Float sums of the accumulator [nrows, W, 3] (host)."""
        out = np.zeros(int(np.prod(self._acc_shape)), np.float32)
        check(self.L.rt_accum_resolve(self._h, None, out.ctypes.data_as(_fp), None), "rt_accum_resolve")
        return out.reshape(self._acc_shape)

    def accum_export(self):
        """(raw int64 fixed-point sums [nrows, W, 3], samples accumulated)."""
        raw = np.zeros(int(np.prod(self._acc_shape)), np.int64)
        done = C.c_int32()
        check(self.L.rt_accum_export(self._h, raw.ctypes.data_as(C.POINTER(C.c_int64)), raw.size, C.byref(done)), "rt_accum_export")
        return raw.reshape(self._acc_shape), done.value

    def accum_import(self, raw, spp_done):
        raw = np.ascontiguousarray(raw, np.int64)
        check(self.L.rt_accum_import(self._h, raw.ctypes.data_as(C.POINTER(C.c_int64)), raw.size, spp_done), "rt_accum_import")

    def progressive(self, cam, W, H, spp, pass_spp, max_depth=50, seed=1984, row0=0, row_step=1, nrows=None,
                    checkpoint=None, on_pass=None):
        """Samples [0, spp) in passes of pass_spp (each a bounded kernel), resuming
        from / saving to `checkpoint` after every pass.  Returns the float sums
        [nrows, W, 3]: bit-identical to render(spp) for any pass split."""
        import os

        nrows = H if nrows is None else nrows
        self.accum_reset(W, nrows)
        sc = self.world.c_struct()
        done = 0
        if checkpoint and os.path.exists(checkpoint):
            n = C.c_int32()
            check(self.L.rt_accum_load(self._h, str(checkpoint).encode(), C.byref(sc), C.byref(cam), W, H, row0, row_step,
                                       nrows, max_depth, seed, C.byref(n)), "rt_accum_load")
            done = n.value
        while done < spp:
            k = min(pass_spp, spp - done)
            self.render_pass(cam, W, H, done, k, max_depth, seed, row0, row_step, nrows)
            done += k
            if checkpoint:
                check(self.L.rt_accum_save(self._h, str(checkpoint).encode(), C.byref(sc), C.byref(cam), H, row0, row_step,
                                           max_depth, seed), "rt_accum_save")
            if on_pass is not None:
                self.synchronize()
                on_pass(done)
        return self.accum_resolve()

    def close(self):
        if self._h:
            self.L.rt_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render(W, H, spp, max_depth, world, cam, seed=1984, device=0):
    """The reference's render surface: image sums [H, W, 3] float32 (row 0 = bottom)."""
    r = Renderer(world, device)
    try:
        return r.render(cam, W, H, spp, max_depth, seed)
    finally:
        r.close()


def render_multi(W, H, spp, max_depth, world, cam, seed=1984, n_gpus=0):
    """Single-process multi-GPU render (interleaved rows + one RCCL gather)."""
    out = np.zeros(W * H * 3, np.float32)
    sc = world.c_struct()
    check(load().rt_render_multi(C.byref(sc), C.byref(cam), W, H, spp, max_depth, seed, n_gpus, out.ctypes.data_as(_fp)), "rt_render_multi")
    return out.reshape(H, W, 3)


class MultiRenderer:
    """rt_multi_*: one context per device with the scene resident and one
    RCCL communicator, reused by every render (include/rtmi.h)."""

    def __init__(self, world, n_gpus=0):
        self.L = load()
        self._h = C.c_void_p()
        sc = world.c_struct()
        check(self.L.rt_multi_create(C.byref(sc), n_gpus, C.byref(self._h)), "rt_multi_create")
        n = C.c_int32()
        check(self.L.rt_multi_device_count(self._h, C.byref(n)), "rt_multi_device_count")
        self.n_gpus = n.value
        self._size = None

    def render(self, cam, W, H, spp, max_depth=50, seed=1984):
        out = np.zeros(W * H * 3, np.float32)
        check(self.L.rt_multi_render(self._h, C.byref(cam), W, H, spp, max_depth, seed, out.ctypes.data_as(_fp)),
              "rt_multi_render")
        return out.reshape(H, W, 3)

    def last_timing(self):
        """(per-device strip ms, gather ms) of the last render / resolve."""
        ms = np.zeros(self.n_gpus, np.float32)
        g = C.c_float()
        check(self.L.rt_multi_last_timing(self._h, ms.ctypes.data_as(_fp), C.byref(g)), "rt_multi_last_timing")
        return ms.tolist(), g.value

    def accum_reset(self, W, H):
        check(self.L.rt_multi_accum_reset(self._h, W, H), "rt_multi_accum_reset")
        self._size = (W, H)

    def render_pass(self, cam, s_begin, s_count, max_depth=50, seed=1984):
        check(self.L.rt_multi_render_pass(self._h, C.byref(cam), s_begin, s_count, max_depth, seed),
              "rt_multi_render_pass")

    def accum_resolve(self):
        W, H = self._size
        out = np.zeros(W * H * 3, np.float32)
        check(self.L.rt_multi_accum_resolve(self._h, out.ctypes.data_as(_fp)), "rt_multi_accum_resolve")
        return out.reshape(H, W, 3)

    def close(self):
        if self._h:
            self.L.rt_multi_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def unpermute_rows(strips, H):
    """rt_unpermute_rows: interleaved strips [G, nrows, W, 3] -> image [H, W, 3]."""
    s = np.ascontiguousarray(strips, np.float32)
    G, nrows, W, _ = s.shape
    out = np.zeros(H * W * 3, np.float32)
    check(load().rt_unpermute_rows(s.ctypes.data_as(_fp), G, nrows, W, H, out.ctypes.data_as(_fp)), "rt_unpermute_rows")
    return out.reshape(H, W, 3)


def quantize(sums, spp):
    """write_color quantisation color.h:14-28 -> uint8 [H, W, 3], top row first."""
    s = np.ascontiguousarray(sums, np.float32)
    H, W, _ = s.shape
    rgb = np.zeros(W * H * 3, np.uint8)
    check(load().rt_quantize(s.ctypes.data_as(_fp), W, H, spp, rgb.ctypes.data_as(C.POINTER(C.c_uint8))), "rt_quantize")
    return rgb.reshape(H, W, 3)


def write_ppm(path, sums, spp, binary=False):
    s = np.ascontiguousarray(sums, np.float32)
    H, W, _ = s.shape
    check(load().rt_write_ppm(path.encode(), s.ctypes.data_as(_fp), W, H, spp, int(binary)), "rt_write_ppm")


def write_pfm(path, sums, spp):
    """PFM of the pre-gamma mean (rt_write_pfm): bottom row first, little-endian."""
    s = np.ascontiguousarray(sums, np.float32)
    H, W, _ = s.shape
    check(load().rt_write_pfm(str(path).encode(), s.ctypes.data_as(_fp), W, H, spp), "rt_write_pfm")


def read_pfm(path):
    """PFM -> float32 [H, W, 3] in file row order (bottom row first), no GPU or library needed."""
    with open(path, "rb") as f:
        tag = f.readline().strip()
        if tag != b"PF":
            raise ValueError(f"{path}: not a colour PFM ({tag!r})")
        W, H = (int(x) for x in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4")
    if data.size != W * H * 3:
        raise ValueError(f"{path}: {data.size} floats for {W}x{H}")
    return data.reshape(H, W, 3).astype(np.float32)
