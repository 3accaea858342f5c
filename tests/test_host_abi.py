"""The C-ABI library on the CPU: it loads, exports every declared symbol, its
host helpers (scene, camera, PPM) equal the reference's, and it refuses to
render without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt
import oracle_py as O
from a_dive_into_ray_tracing_amd import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = O.GOLDEN


def declared_symbols():
    inc = os.path.join(REPO, "include")
    hdr = "".join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith(".h"))
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    L = _abi.load()
    syms = declared_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_abi.SIGNATURES), "ctypes signatures out of sync with include/*.h"


def test_version():
    assert _abi.load().rt_version() == (0 << 16) | 1


def test_scene_random_equals_reference():
    w = rt.random_scene()
    gold = O.load_scene_txt(os.path.join(GOLD, "scene_final.txt"))
    assert len(w) == 487
    assert np.array_equal(w.center_radius.reshape(-1), gold.geom)
    assert np.array_equal(w.mat_kind, gold.kind)
    assert np.array_equal(w.mat_params.reshape(-1), gold.mat)


def test_scene_learn_equals_reference():
    w = rt.learn_scene()
    gold = O.load_scene_txt(os.path.join(GOLD, "scene_learn.txt"))
    assert np.array_equal(w.center_radius.reshape(-1), gold.geom) and np.array_equal(w.mat_kind, gold.kind)
    assert np.array_equal(w.mat_params.reshape(-1), gold.mat)


def test_scene_cap_too_small():
    g, m, k, n = np.zeros(40), np.zeros(40), np.zeros(10, np.int32), C.c_int32()
    rc = _abi.load().rt_scene_random(1, rt._d(g), k.ctypes.data_as(rt._ip), rt._d(m), 10, C.byref(n))
    assert rc == -1 and b"too small" in _abi.load().rt_last_error()


@pytest.mark.parametrize("name", ["final", "learn"])
def test_camera_equals_reference(name):
    cam = rt.final_camera() if name == "final" else rt.learn_camera()
    gold = O.load_camera_txt(os.path.join(GOLD, f"camera_{name}.txt"))
    for k, v in gold.items():
        got = getattr(cam, k)
        assert (list(got) if k != "lens_radius" else got) == v, k


def _write_color_ref(sums, spp):
    """color.h:14-28 in numpy double: int(256*clamp(sqrt(sum/spp),0,0.999))."""
    c = np.sqrt((1.0 / spp) * sums.astype(np.float64))
    return (256 * np.clip(c, 0.0, 0.999)).astype(np.int64)[::-1]


def test_quantize_and_ppm(tmp_path):
    rng = np.random.default_rng(0)
    spp = 37
    sums = (rng.random((9, 13, 3)) * spp * 1.1).astype(np.float32)
    sums[0, 0] = [0, spp, 2 * spp]
    q = rt.quantize(sums, spp)
    assert np.array_equal(q, _write_color_ref(sums, spp))
    p3, p6 = tmp_path / "a.ppm", tmp_path / "b.ppm"
    rt.write_ppm(str(p3), sums, spp)
    rt.write_ppm(str(p6), sums, spp, binary=True)
    tok = p3.read_text().split()
    assert tok[:4] == ["P3", "13", "9", "255"]
    assert np.array_equal(np.array(tok[4:], np.int64).reshape(9, 13, 3), q)
    raw = p6.read_bytes()
    assert raw.startswith(b"P6\n13 9\n255\n") and raw[len(b"P6\n13 9\n255\n"):] == q.tobytes()


def test_ppm_matches_reference_p3_config1():
    """The reference's own P3 of config 1 equals our writer applied to the
    reference's (double) sums rounded to float, except where float rounding
    crosses a quantisation boundary (counted; expected ~0)."""
    scene = O.learn_scene()
    cam = O.learn_camera(400 / 225)
    g = O.OrGlibc()
    O.lib().or_glibc_seed(C.byref(g), 1)
    sums, _ = O.ref_worker(scene, cam, 400, 225, 100, 50, 0, 400 * 225, g)
    q = rt.quantize(sums.reshape(225, 400, 3).astype(np.float32), 100)
    raw = open(os.path.join(GOLD, "learn_400x225x100.ppm"), "rb").read()
    gold = np.frombuffer(raw[len(b"P6\n400 225\n255\n"):], np.uint8).reshape(225, 400, 3)
    diff = np.abs(q.astype(int) - gold.astype(int))
    assert diff.max() <= 1 and (diff > 0).sum() <= 5


def test_render_without_gpu_fails_loudly():
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(rt.RTError) as e:
        rt.render(8, 8, 1, 5, rt.learn_scene(), rt.learn_camera())
    assert "RT_ENODEVICE" in str(e.value)


def test_bad_arguments_rejected():
    L = _abi.load()
    cam = rt.final_camera()
    assert L.rt_render(None, C.byref(cam), 8, 8, 1, 5, 1, None) == -1
    assert L.rt_write_ppm(b"/nonexistent/dir/x.ppm", np.zeros(12, np.float32).ctypes.data_as(rt._fp), 2, 2, 1, 0) == -7
