"""Pin the oracle (oracle/rt_oracle.c, ref mode) to the reference's own outputs.

Every fixture under tests/golden/ was produced by the reference program
itself (oracle/gen_golden.py driving rt_in_one_weekend/ compiled with g++).
The ref-mode restatement must reproduce all of them BIT-EXACTLY, including
the number of rand() draws consumed — this is what licenses the oracle as the
parity checker for the HIP kernel.
"""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

import oracle_py as O

GOLD = O.GOLDEN


def _kats(name):
    lines = open(os.path.join(GOLD, f"kats_{name}.txt")).read().split("\n")
    n, W, H = map(int, lines[0].split())
    out = []
    for line in lines[1 : 1 + n]:
        t = line.split()
        out.append((int(t[0]), int(t[1]), int(t[2]), [float(x) for x in t[3:6]], int(t[6])))
    return W, H, out


def test_glibc_stream_matches_libc():
    """or_glibc restates glibc random_r TYPE_3: compare with libc's own rand()."""
    libc = C.CDLL("libc.so.6")
    for seed in (1, 2, 12345, 4000000000):
        libc.srand(C.c_uint(seed))
        want = [libc.rand() for _ in range(2000)]
        g = O.OrGlibc()
        O.lib().or_glibc_seed(C.byref(g), seed)
        got = [O.lib().or_glibc_rand(C.byref(g)) for _ in range(2000)]
        assert got == want


def test_final_scene_matches_reference():
    sc, _ = O.final_scene()
    gold = O.load_scene_txt(os.path.join(GOLD, "scene_final.txt"))
    assert sc.n == gold.n == 487
    assert np.array_equal(sc.geom, gold.geom)
    assert np.array_equal(sc.kind, gold.kind)
    assert np.array_equal(sc.mat, gold.mat)
    # 394 lambertian / 64 metal / 29 dielectric over all objects
    assert np.bincount(sc.kind).tolist() == [394, 64, 29]


def test_learn_scene_matches_reference():
    sc = O.learn_scene()
    gold = O.load_scene_txt(os.path.join(GOLD, "scene_learn.txt"))
    assert np.array_equal(sc.geom, gold.geom) and np.array_equal(sc.kind, gold.kind) and np.array_equal(sc.mat, gold.mat)


@pytest.mark.parametrize("name", ["final", "learn"])
def test_camera_matches_reference(name):
    cam = O.final_camera() if name == "final" else O.learn_camera()
    gold = O.load_camera_txt(os.path.join(GOLD, f"camera_{name}.txt"))
    got = O.camera_dict(cam)
    for k, v in gold.items():
        assert got[k] == v, k


@pytest.mark.parametrize("name", ["final", "learn"])
def test_seeded_path_kats_bit_exact(name):
    """srand(k) -> one worker() sample -> colour (double, bit-exact) + next rand()."""
    W, H, kats = _kats(name)
    scene = O.load_scene_txt(os.path.join(GOLD, f"scene_{name}.txt"))
    cam = O.final_camera() if name == "final" else O.learn_camera()
    assert len(kats) == 64
    for k, i, j, col, nxt in kats:
        out, got_next = O.ref_kat(scene, cam, W, H, 50, i, j, k)
        assert out.tolist() == col, (k, out, col)
        assert got_next == nxt, k


def test_function_kats_bit_exact():
    lines = open(os.path.join(GOLD, "funcs.txt")).read().split("\n")
    L = O.lib()
    pos = 0

    def section(tag):
        nonlocal pos
        head = lines[pos].split()
        assert head[0] == tag
        n = int(head[1])
        rows = [[float(x) for x in r.split()] for r in lines[pos + 1 : pos + 1 + n]]
        pos += 1 + n
        return rows

    d3 = lambda v: np.ascontiguousarray(v, np.float64)
    n_hit = 0
    for r in section("hit"):
        c, rad, o, d, tmax, h = d3(r[0:3]), r[3], d3(r[4:7]), d3(r[7:10]), r[10], int(r[11])
        t, p, nrm, ff = C.c_double(), np.zeros(3), np.zeros(3), C.c_int32()
        got = L.or_ref_sphere_hit(O.dptr(c), rad, O.dptr(o), O.dptr(d), 0.001, tmax, C.byref(t), O.dptr(p), O.dptr(nrm), C.byref(ff))
        assert got == h
        if h:
            n_hit += 1
            assert t.value == r[12] and p.tolist() == r[13:16] and nrm.tolist() == r[16:19] and ff.value == int(r[19])
    assert n_hit >= 16  # the vectors exercise both outcomes
    for r in section("refract"):
        uv, n, eta = d3(r[0:3]), d3(r[3:6]), r[6]
        out, rf = np.zeros(3), np.zeros(3)
        L.or_ref_refract(O.dptr(uv), O.dptr(n), eta, O.dptr(out))
        L.or_ref_reflect(O.dptr(uv), O.dptr(n), O.dptr(rf))
        cosv = min(-(uv[0] * n[0] + uv[1] * n[1]) - uv[2] * n[2], 1.0)
        assert out.tolist() == r[7:10] and rf.tolist() == r[10:13]
        assert L.or_ref_reflectance(cosv, eta) == r[13]
    for r in section("near_zero"):
        assert L.or_ref_near_zero(O.dptr(d3(r[0:3]))) == int(r[3])
    for r in section("scatter"):
        kind, mat = int(r[0]), d3(r[1:5])
        din, p, nrm, ff = d3(r[5:8]), d3(r[8:11]), d3(r[11:14]), int(r[14])
        ok, att, so, sd = int(r[15]), r[16:19], r[19:22], r[22:25]
        k, nxt = int(r[25]), int(r[26])
        a, o, dd, nx = np.zeros(3), np.zeros(3), np.zeros(3), C.c_int32()
        got = L.or_ref_scatter(kind, O.dptr(mat), O.dptr(din), O.dptr(p), O.dptr(nrm), ff, 1000 + k, O.dptr(a), O.dptr(o), O.dptr(dd), C.byref(nx))
        assert got == ok and a.tolist() == att and o.tolist() == so and dd.tolist() == sd and nx.value == nxt, k


@pytest.mark.parametrize("name,W,H,S,raw", [("final", 24, 16, 8, True), ("learn", 32, 18, 16, True), ("final", 120, 80, 32, False)])
def test_single_threaded_images_bit_exact(name, W, H, S, raw):
    """worker(0, W*H) over the process's own rand() stream: the scene's draws
    first (final), then every sample in reference order."""
    if name == "final":
        scene, g = O.final_scene()
        cam = O.final_camera(W / H)
    else:
        scene = O.learn_scene()
        cam = O.learn_camera(W / H)
        g = O.OrGlibc()
        O.lib().or_glibc_seed(C.byref(g), 1)
    out, draws = O.ref_worker(scene, cam, W, H, S, 50, 0, W * H, g)
    stem = os.path.join(GOLD, f"image_{name}_{W}x{H}x{S}")
    assert hashlib.sha256(out.tobytes()).hexdigest() == open(stem + ".sha256").read().strip()
    if raw:
        assert np.array_equal(out, np.fromfile(stem + ".f64", dtype="<f8"))


@pytest.mark.slow
def test_config1_image_bit_exact():
    """Config 1 (learn, 400x225, 100 spp, depth 50): the whole oracle image."""
    scene = O.learn_scene()
    cam = O.learn_camera(400 / 225)
    g = O.OrGlibc()
    O.lib().or_glibc_seed(C.byref(g), 1)
    out, _ = O.ref_worker(scene, cam, 400, 225, 100, 50, 0, 400 * 225, g)
    assert hashlib.sha256(out.tobytes()).hexdigest() == open(os.path.join(GOLD, "image_learn_400x225x100.sha256")).read().strip()
