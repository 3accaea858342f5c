"""Next-Week renderer — Python view of include/rtmi_nw.h.

Mirrors the reference's rt_next_week/cuda/ vocabulary: a Scene is built with
one call per reference constructor and rendered by the gfx950 kernel; there
is no CPU fallback.

    s = Scene()
    white = s.lambertian(s.solid(.73, .73, .73))           # material.h:40-43
    box = s.translate(s.rotate_y(s.box((0, 0, 0), (165, 330, 165), white), 15), (265, 0, 295))
    s.add(s.constant_medium(box, 0.01, s.solid(0, 0, 0)))   # constant_medium.h
    cam = camera((278, 278, -800), (278, 278, 0), (0, 1, 0), 40, 1.0, 0.0, 800.0)
    sums = NwRenderer(s).render(cam, W, H, spp)

or a reference scene: `s, cam = preset(8, image=earth_rgb, aspect=1.0)`
(create_world main.cu:415-490).
"""
import ctypes as C

import numpy as np

from ._abi import RtNwCamera, RtNwFlat, check, load

__all__ = ["Scene", "NwRenderer", "camera", "preset", "xorwow_uniforms", "load_image", "SCENES"]

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int32)
_u8 = C.POINTER(C.c_uint8)

# create_world's switch cases (main.cu:433-484)
SCENES = {"random": 1, "two_spheres": 2, "two_perlin_spheres": 3, "earth": 4, "simple_light": 5,
          "cornell_box": 6, "cornell_smoke": 7, "final": 8}


def _v3(v):
    return (C.c_double * 3)(*[float(x) for x in v])


def _id(rc, what):
    if rc < 0:
        check(rc, what)
    return rc


def camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, time0=0.0, time1=1.0):
    """camera::camera camera.h:24-62 with the shutter [time0, time1]."""
    cam = RtNwCamera()
    check(load().rt_nw_camera_init(C.byref(cam), _v3(lookfrom), _v3(lookat), _v3(vup), float(vfov), float(aspect),
                                   float(aperture), float(focus_dist), float(time0), float(time1)), "rt_nw_camera_init")
    return cam


class Scene:
    """Host-side scene under construction (rt_nw_scene)."""

    def __init__(self):
        self._h = C.c_void_p()
        check(load().rt_nw_scene_create(C.byref(self._h)), "rt_nw_scene_create")

    # textures texture.h
    def solid(self, r, g, b):
        return _id(load().rt_nw_tex_solid(self._h, r, g, b), "rt_nw_tex_solid")

    def checker(self, even, odd):
        return _id(load().rt_nw_tex_checker(self._h, even, odd), "rt_nw_tex_checker")

    def noise(self, scale, ranvec, perm):
        rv = np.ascontiguousarray(ranvec, np.float32).reshape(256 * 3)
        pm = np.ascontiguousarray(perm, np.int32).reshape(3 * 256)
        return _id(load().rt_nw_tex_noise(self._h, float(scale), rv.ctypes.data_as(_fp), pm.ctypes.data_as(_ip)),
                   "rt_nw_tex_noise")

    def image(self, rgb):
        if rgb is None:
            return _id(load().rt_nw_tex_image(self._h, None, 0, 0), "rt_nw_tex_image")
        a = np.ascontiguousarray(rgb, np.uint8)
        h, w = a.shape[:2]
        return _id(load().rt_nw_tex_image(self._h, a.ctypes.data_as(_u8), w, h), "rt_nw_tex_image")

    # materials material.h
    def lambertian(self, tex):
        return _id(load().rt_nw_mat_lambertian(self._h, tex), "rt_nw_mat_lambertian")

    def metal(self, tex, fuzz):
        return _id(load().rt_nw_mat_metal(self._h, tex, float(fuzz)), "rt_nw_mat_metal")

    def dielectric(self, ir):
        return _id(load().rt_nw_mat_dielectric(self._h, float(ir)), "rt_nw_mat_dielectric")

    def diffuse_light(self, tex):
        return _id(load().rt_nw_mat_diffuse_light(self._h, tex), "rt_nw_mat_diffuse_light")

    def isotropic(self, tex):
        return _id(load().rt_nw_mat_isotropic(self._h, tex), "rt_nw_mat_isotropic")

    # objects
    def sphere(self, center, radius, mat):
        return _id(load().rt_nw_sphere(self._h, _v3(center), float(radius), mat), "rt_nw_sphere")

    def moving_sphere(self, c0, c1, t0, t1, radius, mat):
        return _id(load().rt_nw_moving_sphere(self._h, _v3(c0), _v3(c1), float(t0), float(t1), float(radius), mat),
                   "rt_nw_moving_sphere")

    def rect(self, plane, a0, a1, b0, b1, k, mat):
        """plane 'xy' | 'xz' | 'yz' (aarect.h)."""
        p = {"xy": 0, "xz": 1, "yz": 2}[plane]
        return _id(load().rt_nw_rect(self._h, p, a0, a1, b0, b1, k, mat), "rt_nw_rect")

    def box(self, p0, p1, mat):
        return _id(load().rt_nw_box(self._h, _v3(p0), _v3(p1), mat), "rt_nw_box")

    def constant_medium(self, boundary, density, tex):
        return _id(load().rt_nw_constant_medium(self._h, boundary, float(density), tex), "rt_nw_constant_medium")

    def group(self, objs):
        a = np.ascontiguousarray(objs, np.int32)
        return _id(load().rt_nw_group(self._h, a.ctypes.data_as(_ip), a.size), "rt_nw_group")

    def translate(self, obj, offset):
        return _id(load().rt_nw_translate(self._h, obj, _v3(offset)), "rt_nw_translate")

    def rotate_y(self, obj, angle):
        return _id(load().rt_nw_rotate_y(self._h, obj, float(angle)), "rt_nw_rotate_y")

    def add(self, obj):
        check(load().rt_nw_world_add(self._h, obj), "rt_nw_world_add")
        return self

    def set_background(self, r, g, b):
        check(load().rt_nw_set_background(self._h, r, g, b), "rt_nw_set_background")

    def flat(self):
        """The flattened scene (what the GPU renders), as numpy arrays (copies)."""
        f = RtNwFlat()
        check(load().rt_nw_scene_flat(self._h, C.byref(f)), "rt_nw_scene_flat")

        def arr(p, n, dt=np.float32):
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)

        return {
            "obj": arr(f.obj, 16 * f.n_obj), "inst": arr(f.inst, 8 * f.n_inst), "mat": arr(f.mat, 4 * f.n_mat),
            "tex": arr(f.tex, 8 * f.n_tex), "perlin_vec": arr(f.perlin_vec, 1024 * f.n_perlin),
            "perlin_perm": arr(f.perlin_perm, 768 * f.n_perlin, np.int32),
            "image_desc": arr(f.image_desc, 4 * f.n_image, np.int32),
            "image_px": arr(f.image_px, int(f.image_bytes), np.uint8),
            "background": np.array(list(f.background), np.float32),
            "n_obj": f.n_obj,
        }

    def grid_stats(self):
        """The uniform grid a device context would build (host only,
        rt_nw_scene_grid_stats): {"dims", "max_cell", "n_big", "n_refs"}."""
        dims = (C.c_int32 * 3)()
        mc, nb, nr = C.c_int32(), C.c_int32(), C.c_int32()
        check(load().rt_nw_scene_grid_stats(self._h, dims, C.byref(mc), C.byref(nb), C.byref(nr)),
              "rt_nw_scene_grid_stats")
        return {"dims": tuple(dims), "max_cell": mc.value, "n_big": nb.value, "n_refs": nr.value}

    def close(self):
        if self._h:
            load().rt_nw_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def preset(which, image=None, aspect=1.0, rtl=False):
    """The reference's scene `which` (name or create_world case 1..8) and its camera."""
    w = SCENES.get(which, which)
    s = Scene()
    cam = RtNwCamera()
    if image is not None:
        a = np.ascontiguousarray(image, np.uint8)
        s._img = a
        ptr, ih, iw = a.ctypes.data_as(_u8), a.shape[0], a.shape[1]
    else:
        ptr, ih, iw = None, 0, 0
    check(load().rt_nw_scene_preset(s._h, int(w), ptr, iw, ih, float(aspect), 1 if rtl else 0, C.byref(cam)),
          "rt_nw_scene_preset")
    return s, cam


def xorwow_uniforms(n, seed=1984):
    """curand_init(seed, 0, 0) + n x curand_uniform, restated (the scene generator's stream)."""
    out = np.zeros(n, np.float32)
    check(load().rt_nw_xorwow_uniforms(seed, n, out.ctypes.data_as(_fp)), "rt_nw_xorwow_uniforms")
    return out


def load_image(path):
    """Decode an image file (the earth texture) to h x w x 3 uint8, row 0 at the top (PIL)."""
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGB"), np.uint8)


class NwRenderer:
    """One device context with a resident Next-Week scene (rt_nw_ctx)."""

    def __init__(self, scene, device=0):
        self._h = C.c_void_p()
        check(load().rt_nw_ctx_create(device, C.byref(self._h)), "rt_nw_ctx_create")
        self.set_scene(scene)

    def set_scene(self, scene):
        check(load().rt_nw_ctx_set_scene(self._h, scene._h), "rt_nw_ctx_set_scene")

    def info(self):
        a, b = C.c_int32(), C.c_int32()
        check(load().rt_nw_ctx_info(self._h, C.byref(a), C.byref(b)), "rt_nw_ctx_info")
        return a.value, b.value

    ACCELS = {"auto": 0, "bvh": 1, "grid": 2}

    def set_accel(self, kind):
        """Closest-hit structure: "auto" (the grid when balanced, else the BVH),
        "bvh" or "grid" (rt_nw_ctx_set_accel); the same image either way."""
        check(load().rt_nw_ctx_set_accel(self._h, self.ACCELS[kind]), "rt_nw_ctx_set_accel")

    def accel_info(self):
        """{"accel": the structure renders use, "dims": grid cells per axis
        (zeros: no grid), "max_cell": fullest cell, "n_big": brute-force list}."""
        used, mc, nb = C.c_int32(), C.c_int32(), C.c_int32()
        dims = (C.c_int32 * 3)()
        check(load().rt_nw_ctx_accel_info(self._h, C.byref(used), dims, C.byref(mc), C.byref(nb)),
              "rt_nw_ctx_accel_info")
        names = {v: k for k, v in self.ACCELS.items()}
        return {"accel": names[used.value], "dims": tuple(dims), "max_cell": mc.value, "n_big": nb.value}

    def render(self, cam, W, H, spp, max_depth=50, seed=1984):
        out = np.zeros((H, W, 3), np.float32)
        check(load().rt_nw_render(self._h, C.byref(cam), W, H, spp, max_depth, seed, out.ctypes.data_as(_fp)),
              "rt_nw_render")
        return out

    def render_rows(self, cam, W, H, spp, max_depth, seed, row0, row_step, nrows, dev_ptr, stream=0):
        check(load().rt_nw_render_rows(self._h, C.byref(cam), W, H, spp, max_depth, seed, row0, row_step, nrows,
                                       C.c_void_p(dev_ptr), C.c_void_p(stream)), "rt_nw_render_rows")

    def debug_trace(self, cam, W, H, i, j, s, max_depth=50, seed=1984, cap=64):
        """The segments of one camera sample: rows (o.xyz, d.xyz, t, n.xyz) and (winner index, box face)."""
        rec = np.zeros(12 * cap, np.float32)
        n = C.c_int32()
        check(load().rt_nw_debug_trace(self._h, C.byref(cam), W, H, max_depth, seed, i, j, s, rec.ctypes.data_as(_fp), cap,
                                       C.byref(n)), "rt_nw_debug_trace")
        out = rec[: 12 * n.value].reshape(-1, 12).copy()
        return out[:, [0, 1, 2, 3, 4, 5, 6, 8, 9, 10]], out[:, [7, 11]].view(np.int32)

    def debug_hits(self, rays, keys=None):
        """Closest hit of each ray (rows o.xyz, d.xyz, time) through the walk
        this context renders with: (insertion index or -1, t, box face)."""
        n = len(rays)
        r = np.zeros((n, 8), np.float32)
        r[:, :7] = rays
        k = None if keys is None else np.ascontiguousarray(keys, np.uint64)
        idx, t, face = np.zeros(n, np.int32), np.zeros(n, np.float32), np.zeros(n, np.int32)
        check(load().rt_nw_debug_hits(self._h, r.ctypes.data_as(_fp),
                                      None if k is None else k.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                      idx.ctypes.data_as(_ip), t.ctypes.data_as(_fp), face.ctypes.data_as(_ip)),
              "rt_nw_debug_hits")
        return idx, t, face

    def last_segments(self):
        v = C.c_uint64()
        check(load().rt_nw_ctx_last_segments(self._h, C.byref(v)), "rt_nw_ctx_last_segments")
        return v.value

    def last_kernel(self):
        """Diagnostic: the last render's kernel (rt_nw_ctx_last_kernel)."""
        v = (C.c_int32 * 4)()
        check(load().rt_nw_ctx_last_kernel(self._h, v), "rt_nw_ctx_last_kernel")
        return dict(zip(("persistent", "grid", "spheres_only", "chunk"), list(v)))

    def close(self):
        if self._h:
            load().rt_nw_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
