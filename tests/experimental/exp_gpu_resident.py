"""The resident grid kernel (RT_KERNEL_RESIDENT) against the
oracle and the grid kernel, bit for bit — on the experimental build
(lib/librtmi_experimental.so), run by tests/test_gpu_experimental.py in a
child process.

Its waves take work items from a global counter, so which wave renders which
item changes from run to run; the per-pixel sums are integers flushed per
item (global atomics, or the floats when an item covers its whole tile), so
the image may not.  These tests pin that: small images against the oracle's
fast mode (edge tiles, 1 spp, depth 1-2, whole-tile and chunked items), the
learn scene, config 2 and interleaved strips of it against the grid kernel's
frame with the same world.hit count, progressive passes, every accelerated
closest-hit kind (the grid in LDS and in global memory, the BVH), a scene of
3 000 spheres, and repeated renders.
"""
import ctypes as C

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt
import oracle_py as O

pytestmark = pytest.mark.gpu
SEED = 1984
RESIDENT = 3  # last_schedule()["persistent"] of a resident launch


@pytest.fixture(scope="module")
def world():
    return rt.random_scene()


@pytest.fixture(scope="module")
def res_renderer(world):
    r = rt.Renderer(world, 0)
    r.set_accel("grid")
    r.set_kernel("resident")
    yield r
    r.close()


def o_cam(cam):
    c = O.OrCamera()
    C.memmove(C.byref(c), C.byref(cam), C.sizeof(c))
    return c


def o_scene(w):
    return O.Scene(w.center_radius, w.mat_kind, w.mat_params)


@pytest.mark.parametrize("W,H,S,depth,tile_w,chunk", [
    (48, 32, 8, 50, 0, 0), (37, 23, 5, 50, 8, 0), (64, 36, 16, 50, 16, 0), (20, 11, 3, 1, 8, 0),
    (16, 16, 4, 2, 0, 0), (9, 7, 1, 50, 0, 0), (80, 48, 24, 50, 8, 5), (120, 80, 64, 50, 0, 0),
    (40, 24, 30, 50, 8, 30), (33, 17, 7, 50, 16, 3)])
def test_resident_bit_exact_vs_oracle(W, H, S, depth, tile_w, chunk, world, res_renderer):
    cam = rt.final_camera(W / H)
    res_renderer.set_tuning(tile_w, chunk)
    try:
        got = res_renderer.render(cam, W, H, S, depth, SEED)
        sch = res_renderer.last_schedule()
        segs = res_renderer.last_segments()
    finally:
        res_renderer.set_tuning(0, 0)
    assert sch["persistent"] == RESIDENT and sch["bvh"] == 2, sch  # the resident kernel ran, through the grid
    want = O.fast_render(o_scene(world), o_cam(cam), W, H, S, depth, SEED)
    assert np.array_equal(got, want), np.abs(got - want).max()
    assert segs == O.fast_segments(o_scene(world), o_cam(cam), W, H, S, depth, SEED)


def test_resident_whole_tile_items_write_floats(world, res_renderer):
    """chunk = spp: one item per tile, which the wave writes as floats
    (no accumulator, no finalize) — the same bits."""
    W, H, S = 72, 40, 6
    cam = rt.final_camera(W / H)
    res_renderer.set_tuning(8, S)
    try:
        got = res_renderer.render(cam, W, H, S, 50, SEED)
        sch = res_renderer.last_schedule()
    finally:
        res_renderer.set_tuning(0, 0)
    assert sch["persistent"] == RESIDENT and sch["items_per_tile"] == 1 and sch["block_flush"] == 1, sch
    assert np.array_equal(got, O.fast_render(o_scene(world), o_cam(cam), W, H, S, 50, SEED))


def test_resident_learn_scene_vs_oracle():
    """The learn() scene (5 spheres, a hollow negative-radius sphere)."""
    w = rt.learn_scene()
    r = rt.Renderer(w, 0)
    try:
        r.set_kernel("resident")
        cam = rt.learn_camera(64 / 36)
        got = r.render(cam, 64, 36, 16, 50, SEED)
    finally:
        r.close()
    assert np.array_equal(got, O.fast_render(o_scene(w), o_cam(cam), 64, 36, 16, 50, SEED))


@pytest.fixture(scope="module")
def grid_frame(world):
    r = rt.Renderer(world, 0)
    try:
        r.set_accel("grid")
        r.set_kernel("grid")
        img = r.render(rt.final_camera(1.5), 1200, 800, 500, 50, SEED)
        segs = r.last_segments()
        assert r.last_schedule()["persistent"] == 0
    finally:
        r.close()
    return img, segs


def test_resident_config2_equals_grid_kernel(grid_frame, res_renderer):
    """Config 2 (1200x800x500): the grid kernel's frame bit for bit, with the
    same number of world.hit calls; twice (the second render dispatches by
    the first one's cost map)."""
    img, segs = grid_frame
    for _ in range(2):
        got = res_renderer.render(rt.final_camera(1.5), 1200, 800, 500, 50, SEED)
        assert res_renderer.last_schedule()["persistent"] == RESIDENT
        assert res_renderer.last_segments() == segs
        assert np.array_equal(got, img)


@pytest.mark.parametrize("G,g", [(8, 3), (3, 2), (8, 7)])
def test_resident_strip_equals_frame_rows(G, g, grid_frame, res_renderer):
    """One rank's interleaved strip equals those rows of the frame; padded
    rows stay zero."""
    torch = pytest.importorskip("torch")
    img, _ = grid_frame
    W, H, S = 1200, 800, 500
    nrows = (H + G - 1) // G
    strip = torch.full((nrows, W, 3), -1.0, dtype=torch.float32, device="cuda:0")
    res_renderer.render_rows(rt.final_camera(1.5), W, H, S, 50, SEED, g, G, nrows, strip.data_ptr(), 0)
    res_renderer.synchronize()
    sch = res_renderer.last_schedule()
    assert sch["persistent"] == RESIDENT and sch["items_per_tile"] > 1, sch
    s = strip.cpu().numpy()
    nvalid = len(range(g, H, G))
    assert np.array_equal(s[:nvalid], img[g::G])
    assert not s[nvalid:].any()


def test_resident_progressive_passes(world, res_renderer):
    W, H = 96, 64
    cam = rt.final_camera(W / H)
    want = O.fast_render(o_scene(world), o_cam(cam), W, H, 12, 50, SEED)
    res_renderer.accum_reset(W, H)
    for s0, n in ((0, 5), (5, 1), (6, 6)):
        res_renderer.render_pass(cam, W, H, s0, n)
        assert res_renderer.last_schedule()["persistent"] == RESIDENT
    assert np.array_equal(res_renderer.accum_resolve(), want)


@pytest.mark.parametrize("accel,env,kind", [("bvh", None, 1), ("grid", "RTMI_GRID_GLOBAL", 4),
                                            ("bvh", "RTMI_BVH_GLOBAL", 1)])
def test_resident_other_closest_hit_kinds(accel, env, kind, world, monkeypatch):
    """The BVH in LDS, the grid and the BVH walked in global memory (forced on
    the final scene): the oracle's image and world.hit count."""
    if env:
        monkeypatch.setenv(env, "1")  # (read when the context is created)
    W, H, S = 64, 40, 6
    cam = rt.final_camera(W / H)
    r = rt.Renderer(world, 0)
    try:
        r.set_accel(accel)
        r.set_kernel("resident")
        got = r.render(cam, W, H, S, 50, SEED)
        sch, segs = r.last_schedule(), r.last_segments()
    finally:
        r.close()
    assert sch["persistent"] == RESIDENT and sch["bvh"] == kind, sch
    assert np.array_equal(got, O.fast_render(o_scene(world), o_cam(cam), W, H, S, 50, SEED))
    assert segs == O.fast_segments(o_scene(world), o_cam(cam), W, H, S, 50, SEED)


def test_resident_large_scene_vs_oracle():
    """3 000 spheres: the grid walked in global memory (over the LDS budget)."""
    n = 3000
    g = np.random.default_rng(n)
    c = np.column_stack([g.uniform(-40, 40, n), g.uniform(0.05, 0.3, n), g.uniform(-40, 40, n)])
    rad = g.uniform(0.03, 0.2, n)
    kinds = g.integers(0, 3, n).astype(np.int32)
    params = np.column_stack([g.uniform(0.1, 0.9, (n, 3)), np.where(kinds == 2, 1.5, g.uniform(0, 0.5, n))])
    cr = np.vstack([[0, -1000, 0, 1000], np.column_stack([c, rad])])
    kinds = np.concatenate([[0], kinds]).astype(np.int32)
    params = np.vstack([[0.5, 0.5, 0.5, 0], params])
    world = rt.World(cr, kinds, params)
    W, H, S = 24, 16, 2
    cam = rt.camera((20, 3, 12), (0, 0, 0), (0, 1, 0), 30.0, W / H, 0.05, 20.0)
    r = rt.Renderer(world, 0)
    try:
        r.set_accel("grid")
        r.set_kernel("resident")
        got = r.render(cam, W, H, S, 50, SEED)
        sch, segs = r.last_schedule(), r.last_segments()
    finally:
        r.close()
    assert sch["persistent"] == RESIDENT and sch["bvh"] == 4, sch
    assert np.array_equal(got, O.fast_render(o_scene(world), o_cam(cam), W, H, S, 50, SEED))
    assert segs == O.fast_segments(o_scene(world), o_cam(cam), W, H, S, 50, SEED)


def test_resident_repeated_renders_are_identical(res_renderer):
    """Which wave takes which item differs run to run; the image may not."""
    cam = rt.final_camera(1.5)
    a = res_renderer.render(cam, 300, 200, 64, 50, SEED)
    for _ in range(3):
        assert np.array_equal(res_renderer.render(cam, 300, 200, 64, 50, SEED), a)
