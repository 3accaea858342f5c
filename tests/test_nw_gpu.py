"""Next-Week renderer on the GPU: the gfx950 kernel
(librtmi.so rt_nw_*) against the CPU oracle (oracle/rt_nw_oracle.inc).

  * bit-exact: every reference scene (create_world cases 1-8), ragged sizes,
    strips and chunked accumulation give the oracle's sums bit for bit and
    the same world.hit count — the GPU's object BVH and leaf order against
    the oracle's brute-force list;
  * statistics: the final scene (main.cu:331-413) at the reference's
    800x800 against the reference's own 5000-spp render,
    gallery/final_scene_5000.png (tests/golden/), by 50x50-pixel tile means.
"""
import os
import time

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd.nextweek as nw
import oracle_py as O

pytestmark = pytest.mark.gpu
GOLD = O.GOLDEN
SEED = 1984


@pytest.fixture(scope="module")
def earth():
    return nw.load_image(os.path.join(GOLD, "earthmap.jpeg"))


@pytest.mark.parametrize("accel", ["bvh", "grid"])
@pytest.mark.parametrize("which", list(range(1, 9)))
def test_presets_bit_exact_vs_oracle(which, accel, earth):
    """Both closest-hit structures (the BVH and the uniform grid with its
    brute-force list) against the oracle's plain list."""
    W, H, spp = 29, 23, 3  # ragged: partial 8x8 tiles on both axes
    s, cam = nw.preset(which, image=earth, aspect=W / H)
    r = nw.NwRenderer(s)
    r.set_accel(accel)
    info = r.accel_info()
    if accel == "grid" and which == 1:
        assert info["accel"] == "grid" and info["n_big"] >= 1, info  # the R = 1000 ground beside the grid
    got = r.render(cam, W, H, spp, 50, SEED)
    segs = r.last_segments()
    r.close()
    want, want_segs = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED)
    assert np.isfinite(got).all()
    assert np.array_equal(got, want), f"scene {which}: max |d| {np.abs(got - want).max()}"
    assert segs == want_segs


@pytest.mark.parametrize("accel", ["bvh", "grid"])
@pytest.mark.parametrize("which", [1, 6, 7, 8])
def test_chunked_strips_bit_exact(which, accel, earth):
    """spp > the 32-sample item (two-item accumulation + finalize) and an
    interleaved strip of rows, through rt_nw_render_rows on a torch stream."""
    import torch

    W, H, spp = 24, 40, 70
    s, cam = nw.preset(which, image=earth, aspect=1.0)
    r = nw.NwRenderer(s)
    r.set_accel(accel)
    row0, step, nrows = 1, 3, 14  # rows 1, 4, ..., 40 (the last past H: zero)
    strip = torch.full((nrows, W, 3), -1.0, dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()
    r.render_rows(cam, W, H, spp, 50, SEED, row0, step, nrows, strip.data_ptr(), st.cuda_stream)
    st.synchronize()
    got = strip.cpu().numpy()
    r.close()
    want, _ = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED, row0=row0, row_step=step, nrows=13)
    assert np.array_equal(got[:13], want)
    assert (got[13] == 0).all()


def test_depth_limit_returns_background(earth):
    """max_depth 1: every path that scatters once returns the background
    (main.cu:100); sky scenes show it."""
    s, cam = nw.preset(2, aspect=1.0)  # two_spheres, sky background
    r = nw.NwRenderer(s)
    got = r.render(cam, 16, 16, 4, 1, SEED)
    r.close()
    want, _ = O.nw_render(s.flat(), cam, 16, 16, 4, 1, SEED)
    assert np.array_equal(got, want)


def _png(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGB"), dtype=np.float64)


def _quantize(sums, spp):
    """main.cu:563-575 (255.99 * sqrt(mean), clamped to a byte as a PNG holds it), top row first."""
    c = np.sqrt(np.clip(sums / spp, 0, None))
    return np.clip(np.floor(255.99 * c), 0, 255)[::-1]


def test_final_scene_statistics_vs_reference_gallery(earth):
    """The final scene at 800x800 (main.cu:520-523) vs the reference's own
    render at 5000 spp, by 50x50-pixel tile means (printed for the record).
    What remains is our 1024-spp noise and the deviations of DESIGN.md §9
    (our sample stream vs per-pixel curand, the JPEG decoder)."""
    W = H = 800
    spp = 1024
    s, cam = nw.preset("final", image=earth, aspect=1.0)
    r = nw.NwRenderer(s)
    t0 = time.time()
    img = r.render(cam, W, H, spp, 50, SEED)
    dt = time.time() - t0
    segs = r.last_segments()
    r.close()
    ours = _quantize(img, spp)
    ref = _png(os.path.join(GOLD, "gallery_final_scene_5000.png"))
    d = ours - ref
    to = ours.reshape(16, 50, 16, 50, 3).mean(axis=(1, 3))
    tr = ref.reshape(16, 50, 16, 50, 3).mean(axis=(1, 3))
    td = np.abs(to - tr)
    print(f"nw final 800x800x{spp}: {dt:.2f} s, {W * H * spp / dt / 1e6:.0f} Msamples/s, {segs / (W * H * spp):.3f} seg/sample; "
          f"vs gallery: bias {d.mean():.3f} MAE {np.abs(d).mean():.3f} tile MAE {td.mean():.3f} tile max {td.max():.2f} "
          f"tile p95 {np.percentile(td, 95):.2f}")
    # measured at 1024 spp: bias -0.55, tile MAE 0.59 (before the medium rules of
    # bias -12.7, tile MAE 12.9)
    assert abs(d.mean()) < 1.0 and td.mean() < 1.0 and td.max() < 6


def test_cli_matches_library(tmp_path, earth):
    """bin/rtmi_nw_render (main.cu main() as a driver): its P3 is the library's
    sums quantised as main.cu:567-575 (unclamped), scene by name or number."""
    import subprocess

    from PIL import Image

    exe = os.path.join(os.path.dirname(nw.__file__), "bin", "rtmi_nw_render")
    tex = tmp_path / "earth.ppm"
    Image.fromarray(earth).save(tex)
    W, H, spp = 24, 16, 4
    for scene, which in (("final", 8), ("5", 5)):
        out = tmp_path / f"o{which}.ppm"
        subprocess.run([exe, "--scene", scene, "--width", str(W), "--height", str(H), "--spp", str(spp),
                        "--texture", str(tex), "--out", str(out)], check=True, capture_output=True, timeout=120)
        tok = out.read_text().split()
        assert tok[:4] == ["P3", str(W), str(H), "255"]
        got = np.array(tok[4:], np.int64).reshape(H, W, 3)
        s, cam = nw.preset(which, image=earth, aspect=W / H)
        r = nw.NwRenderer(s)
        sums = r.render(cam, W, H, spp, 50, SEED)
        r.close()
        mean = (sums / np.float32(spp)).astype(np.float32)
        want = np.floor(255.99 * np.sqrt(mean).astype(np.float32).astype(np.float64)).astype(np.int64)[::-1]
        assert np.array_equal(got, want)


@pytest.mark.parametrize("accel", ["bvh", "grid"])
@pytest.mark.parametrize("shutter", [(0.0, 1.0), (0.3, 0.6)])
def test_moving_spheres_bit_exact(shutter, accel):
    """Moving spheres with their own time ranges inside and outside the
    shutter (the centre extrapolates linearly; their BVH boxes are swept over
    [0, 1]), under translate/rotate_y instances and as a medium's boundary:
    equal to the oracle (brute force), world.hit counts included."""
    g = np.random.default_rng(7)
    s = nw.Scene()
    gray = s.lambertian(s.solid(0.5, 0.5, 0.5))
    s.add(s.sphere((0, -1000, 0), 1000, gray))
    kids = []
    for k in range(150):
        c0 = (g.uniform(-6, 6), g.uniform(0.1, 1.5), g.uniform(-6, 6))
        c1 = (c0[0] + g.uniform(-1, 1), c0[1] + g.uniform(0, 1.2), c0[2] + g.uniform(-1, 1))
        t0, t1 = [(0.0, 1.0), (0.2, 0.7), (-0.5, 0.5), (0.4, 2.0)][k % 4]
        mat = [gray, s.metal(s.solid(0.8, 0.7, 0.6), 0.2), s.dielectric(1.5)][k % 3]
        obj = s.moving_sphere(c0, c1, t0, t1, g.uniform(0.1, 0.4), mat)
        if k % 5 == 0:
            kids.append(obj)  # instanced below
        else:
            s.add(obj)
    inst = s.translate(s.rotate_y(s.group(kids), 25.0), (1.0, 0.2, -0.5))
    s.add(inst)
    fog = s.constant_medium(s.moving_sphere((2, 1, 2), (2, 1.5, 2.5), 0.0, 1.0, 0.8, gray), 0.5, s.solid(0.9, 0.9, 0.9))
    s.add(fog)
    s.add(s.box((-2, 0, -2), (-1, 1, -1), gray))
    s.set_background(0.7, 0.8, 1.0)
    W, H, spp = 40, 30, 6
    cam = nw.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 30.0, W / H, 0.1, 10.0, *shutter)
    r = nw.NwRenderer(s)
    r.set_accel(accel)
    assert r.accel_info()["accel"] == accel
    got, segs = r.render(cam, W, H, spp, 50, SEED), r.last_segments()
    r.close()
    want, want_segs = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED)
    assert np.array_equal(got, want), f"max |d| {np.abs(got - want).max()}"
    assert segs == want_segs


@pytest.mark.parametrize("seed", [3, 11])
def test_grid_mixed_objects_bit_exact(seed):
    """The grid over every object kind at once — rectangles (zero thickness)
    in the three planes, boxes, rotated and translated instances, moving and
    static spheres, a box-bounded medium, lights — scaled x100 and shifted
    far from the origin (coordinates ~3000: cell faces far from 0 in float):
    grid == oracle (brute force) and BVH == oracle, world.hit counts
    included; auto picks the grid."""
    g = np.random.default_rng(seed)
    S = 100.0
    off = np.array([3000.0, -1500.0, 2200.0])
    s = nw.Scene()
    gray = s.lambertian(s.solid(0.5, 0.5, 0.5))
    mats = [gray, s.metal(s.solid(0.8, 0.7, 0.6), 0.1), s.dielectric(1.5)]
    light = s.diffuse_light(s.solid(4, 4, 4))
    s.add(s.sphere(tuple(off + S * np.array([0, -1000, 0])), 1000 * S, gray))
    kids = []
    for k in range(240):
        inside = k % 8 == 0  # every 8th object goes into the instance: built around the origin, moved by it
        base = np.zeros(3) if inside else off
        P = lambda *v: tuple(base + S * np.array(v, dtype=np.float64))
        x, y, z = g.uniform(-8, 8), g.uniform(0.1, 2.0), g.uniform(-8, 8)
        m = mats[k % 3]
        kind = k % 6
        if kind == 0:
            o = s.sphere(P(x, y, z), S * g.uniform(0.1, 0.4), m)
        elif kind == 1:
            o = s.moving_sphere(P(x, y, z), P(x, y + g.uniform(0, 0.5), z), 0.0, 1.0, S * g.uniform(0.1, 0.3), m)
        elif kind == 2:
            o = s.box(P(x, 0, z), P(x + g.uniform(0.2, 0.8), g.uniform(0.2, 1.5), z + g.uniform(0.2, 0.8)), m)
        else:
            plane = kind - 3  # xy, xz, yz: in-plane axes (a, b), plane axis k
            ax_a, ax_b, ax_k = [0, 0, 1][plane], [1, 2, 2][plane], [2, 1, 0][plane]
            lo = np.array(P(x, y, z))
            o = s.rect(["xy", "xz", "yz"][plane], lo[ax_a], lo[ax_a] + 0.6 * S, lo[ax_b], lo[ax_b] + 0.6 * S,
                       float(lo[ax_k]), m if k % 7 else light)
        if inside:
            kids.append(o)
        else:
            s.add(o)
    s.add(s.translate(s.rotate_y(s.group(kids), 33.0), tuple(off + S * np.array([0.5, 0.0, -0.7]))))
    fog_box = s.box(tuple(off + S * np.array([3, 0, 3])), tuple(off + S * np.array([4.5, 1.5, 4.5])), gray)
    s.add(s.constant_medium(fog_box, 0.008, s.solid(0.9, 0.9, 0.9)))
    s.set_background(0.7, 0.8, 1.0)
    stats = s.grid_stats()
    assert stats["n_big"] == 1 and stats["max_cell"] <= 24, stats
    W, H, spp = 40, 30, 5
    cam = nw.camera(tuple(off + S * np.array([13, 2, 3])), tuple(off), (0, 1, 0), 30.0, W / H, 0.1 * S, 10.0 * S)
    r = nw.NwRenderer(s)
    assert r.accel_info()["accel"] == "grid"
    got, segs = r.render(cam, W, H, spp, 50, SEED), r.last_segments()
    r.set_accel("bvh")
    got_bvh = r.render(cam, W, H, spp, 50, SEED)
    r.close()
    want, want_segs = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED)
    assert np.array_equal(got, want), f"max |d| {np.abs(got - want).max()}"
    assert np.array_equal(got_bvh, want)
    assert segs == want_segs


@pytest.mark.parametrize("which", [1, 2])
@pytest.mark.parametrize("size", [(29, 23, 3), (64, 40, 70)])
def test_spheres_only_kernel_bit_exact(which, size, monkeypatch, earth):
    """Spheres-only scenes (spheres and moving spheres, solid and checker
    textures, no instances or media) take the persistent grid kernel's
    spheres-only instantiation (the other kinds' code compiled out); its image
    and world.hit count equal the oracle's and the general kernel's
    (RTMI_NW_SIMPLE=0), bit for bit.  70 spp: several items per pixel."""
    W, H, spp = size
    s, cam = nw.preset(which, image=earth, aspect=W / H)
    imgs, segs = [], []
    for simple in ("1", "0"):
        monkeypatch.setenv("RTMI_NW_SIMPLE", simple)
        r = nw.NwRenderer(s)
        try:
            r.set_accel("grid")
            imgs.append(r.render(cam, W, H, spp, 50, SEED))
            segs.append(r.last_segments())
            k = r.last_kernel()
        finally:
            r.close()
        assert k["persistent"] == 1 and k["grid"] == 1 and k["spheres_only"] == int(simple == "1"), k
    want, want_segs = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED)
    assert np.array_equal(imgs[0], want), f"max |d| {np.abs(imgs[0] - want).max()}"
    assert np.array_equal(imgs[1], want)
    assert segs[0] == segs[1] == want_segs


def test_spheres_only_moving_and_not_simple_scenes():
    """Moving spheres with their own time ranges (inside and outside the
    shutter) and a checker texture on the spheres-only kernel, bit-exact vs the
    oracle; a scene with one rectangle, or a checker of an image texture, stays
    on the general kernel."""
    g = np.random.default_rng(5)
    s = nw.Scene()
    check = s.lambertian(s.checker(s.solid(0.2, 0.3, 0.1), s.solid(0.9, 0.9, 0.9)))
    s.add(s.sphere((0, -1000, 0), 1000, check))
    for k in range(120):
        c0 = (g.uniform(-6, 6), g.uniform(0.1, 1.5), g.uniform(-6, 6))
        c1 = (c0[0] + g.uniform(-1, 1), c0[1] + g.uniform(0, 1.2), c0[2] + g.uniform(-1, 1))
        t0, t1 = [(0.0, 1.0), (0.2, 0.7), (-0.5, 0.5), (0.4, 2.0)][k % 4]
        mat = [check, s.metal(s.solid(0.8, 0.7, 0.6), 0.2), s.dielectric(1.5), s.diffuse_light(s.solid(4, 4, 4))][k % 4]
        s.add(s.moving_sphere(c0, c1, t0, t1, g.uniform(0.1, 0.4), mat) if k % 2 else
              s.sphere(c0, g.uniform(0.1, 0.4), mat))
    s.set_background(0.7, 0.8, 1.0)
    W, H, spp = 40, 30, 6
    cam = nw.camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 30.0, W / H, 0.1, 10.0, 0.3, 0.6)
    r = nw.NwRenderer(s)
    r.set_accel("grid")
    got, segs, k = r.render(cam, W, H, spp, 50, SEED), r.last_segments(), r.last_kernel()
    r.close()
    assert k["spheres_only"] == 1, k
    want, want_segs = O.nw_render(s.flat(), cam, W, H, spp, 50, SEED)
    assert np.array_equal(got, want), f"max |d| {np.abs(got - want).max()}"
    assert segs == want_segs
    for extra in ("rect", "image"):
        s2, _ = nw.preset(2, aspect=W / H)
        if extra == "rect":
            s2.add(s2.rect("xy", -1, 1, -1, 1, -3, s2.lambertian(s2.solid(0.5, 0.5, 0.5))))
        else:  # a checker with an image leaf (the missing-image texture)
            s2.add(s2.sphere((0, 5, 0), 1, s2.lambertian(s2.checker(s2.image(None), s2.solid(1, 1, 1)))))
        r = nw.NwRenderer(s2)
        r.set_accel("grid")
        r.render(cam, W, H, 2, 50, SEED)
        k = r.last_kernel()
        r.close()
        assert k["spheres_only"] == 0, (extra, k)


_TRACE_CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["RTMI_REPO"])
import a_dive_into_ray_tracing_amd.nextweek as nw
img = nw.load_image(os.path.join(os.environ["RTMI_REPO"], "tests", "golden", "earthmap.jpeg"))
out = {}
for which in (1, 8):
    s, cam = nw.preset(which, image=img, aspect=1.0)
    r = nw.NwRenderer(s)
    for (i, j) in ((3, 5), (12, 9)):
        f, k = r.debug_trace(cam, 16, 16, i, j, 2)
        out[f"f{which}_{i}_{j}"], out[f"k{which}_{i}_{j}"] = f, k
    r.close()
np.savez(sys.argv[1], **out)
"""


@pytest.mark.parametrize("lib", ["librtmi_stats.so"])
def test_debug_trace_on_the_stats_build(lib, tmp_path):
    """rt_nw_debug_trace runs on the RTMI_STATS build too (its trace kernel
    hands the walk a counter of its own: ADVICE r03 found a null counter
    pointer there), and records the same segments as the product library."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for name in ("librtmi.so", lib):
        env = dict(os.environ, RTMI_REPO=root, RTMI_LIBRARY=os.path.join(root, "a_dive_into_ray_tracing_amd", "lib", name))
        p = subprocess.run([sys.executable, "-c", _TRACE_CHILD, str(tmp_path / name)], env=env, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        res[name] = np.load(str(tmp_path / name) + ".npz")
    a, b = res["librtmi.so"], res[lib]
    assert sorted(a.files) == sorted(b.files)
    for key in a.files:
        assert a[key].shape[0] >= 1
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize("accel", ["grid", "bvh"])
@pytest.mark.parametrize("which", [1, 8])
def test_walks_with_signed_zero_directions_equal_brute_force(which, accel, earth):
    """ADVICE r04 / VERDICT r05 item 6: rays whose direction has exact +0.0
    and -0.0 components (and axis-aligned rays, two zero components) through
    the Next-Week grid walk and the BVH walk (rt_nw_debug_hits: the walk the
    renders use) give the oracle's brute-force closest hit — insertion
    index, t and box face — bit for bit.  The grid walk takes its step
    directions from the culling inverses, because safe_inv maps -0.0 to
    -1e20 (rtmi_nw_path.h hit_world_nw_grid): a `d >= 0` test would step a
    -0.0 axis the wrong way.  Scenes: the motion-blur random scene (moving
    spheres, shutter times) and the final scene (boxes, instances, media
    with their segment keys)."""
    g = np.random.default_rng(100 + which)
    s, _ = nw.preset(which, image=earth, aspect=1.0)
    n = 200_000 if which == 1 else 60_000
    if which == 1:
        lo, hi = np.array([-13.0, -0.2, -13.0]), np.array([13.0, 3.0, 13.0])
    else:
        lo, hi = np.array([-50.0, -20.0, -650.0]), np.array([650.0, 600.0, 650.0])
    o = lo + (hi - lo) * g.random((n, 3))
    d = g.normal(size=(n, 3))
    z = g.random((n, 3)) < 0.06
    d[z] = np.where(g.random(int(z.sum())) < 0.5, 0.0, -0.0)  # exact zeros of both signs
    ax = g.random(n) < 0.1  # axis-aligned: one non-zero component, the others signed zeros
    k = g.integers(0, 3, int(ax.sum()))
    dd = np.where(g.random((int(ax.sum()), 3)) < 0.5, 0.0, -0.0)
    dd[np.arange(dd.shape[0]), k] = np.where(g.random(dd.shape[0]) < 0.5, 1.0, -1.0)
    d[ax] = dd
    d[np.all(d == 0, axis=1)] = [0.0, -1.0, -0.0]  # (not a ray)
    t = g.random(n)
    rays = np.column_stack([o, d, t]).astype(np.float32)
    assert np.signbit(rays[:, 3:6][rays[:, 3:6] == 0]).mean() > 0.3  # -0.0 present
    keys = g.integers(0, 2**63, n, dtype=np.uint64)
    r = nw.NwRenderer(s)
    try:
        r.set_accel(accel)
        assert r.accel_info()["accel"] == accel
        got = r.debug_hits(rays, keys)
    finally:
        r.close()
    want = O.nw_hits(s.flat(), rays, keys)
    assert (want[0] >= 0).mean() > 0.2  # the rays hit things
    for name, a, b in zip(("index", "t", "face"), got, want):
        bad = np.nonzero(a != b)[0]
        assert bad.size == 0, f"{name}: {bad.size} rays differ, first {bad[:5]}: {a[bad[:5]]} vs {b[bad[:5]]}"
