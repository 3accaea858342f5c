"""The queue kernel (RT_KERNEL_QUEUE) against the oracle and
the other kernels, bit for bit — on the experimental build
(lib/librtmi_experimental.so: `make -C a_dive_into_ray_tracing_amd/csrc
experimental`), run by tests/test_gpu_experimental.py in a child process.

Rays migrate between the waves of a block through the LDS pool and end in
whichever wave holds them; the per-pixel sums are integers, so every order
gives the same bits.  These tests pin that: small images against the
oracle's fast mode (edge tiles, 1 spp, depth 1-2, the whole-tile and the
chunked item paths), config 2 and strips of it against the grid kernel's
frame, progressive passes, and the reference's world.hit count.
"""
import ctypes as C

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt
import oracle_py as O

pytestmark = pytest.mark.gpu
SEED = 1984


@pytest.fixture(scope="module")
def world():
    return rt.random_scene()


@pytest.fixture(scope="module")
def queue_renderer(world):
    r = rt.Renderer(world, 0)
    r.set_accel("grid")
    r.set_kernel("queue")
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
    (16, 16, 4, 2, 0, 0), (9, 7, 1, 50, 0, 0), (80, 48, 24, 50, 8, 5), (120, 80, 64, 50, 0, 0)])
def test_queue_bit_exact_vs_oracle(W, H, S, depth, tile_w, chunk, world, queue_renderer):
    cam = rt.final_camera(W / H)
    queue_renderer.set_tuning(tile_w, chunk)
    try:
        got = queue_renderer.render(cam, W, H, S, depth, SEED)
        sch = queue_renderer.last_schedule()
    finally:
        queue_renderer.set_tuning(0, 0)
    assert sch["persistent"] == 2 and sch["bvh"] == 2, sch  # the queue kernel ran, through the grid
    want = O.fast_render(o_scene(world), o_cam(cam), W, H, S, depth, SEED)
    assert np.array_equal(got, want), np.abs(got - want).max()


def test_queue_learn_scene_vs_oracle():
    """The learn() scene (5 spheres: a hollow negative-radius sphere, grid or
    brute force as the scene allows) through the queue kernel."""
    w = rt.learn_scene()
    r = rt.Renderer(w, 0)
    try:
        r.set_kernel("queue")
        cam = rt.learn_camera(64 / 36)
        got = r.render(cam, 64, 36, 16, 50, SEED)
    finally:
        r.close()
    want = O.fast_render(o_scene(w), o_cam(cam), 64, 36, 16, 50, SEED)
    assert np.array_equal(got, want)


@pytest.fixture(scope="module")
def grid_frame(world):
    r = rt.Renderer(world, 0)
    try:
        r.set_accel("grid")
        img = r.render(rt.final_camera(1.5), 1200, 800, 500, 50, SEED)
        segs = r.last_segments()
    finally:
        r.close()
    return img, segs


def test_queue_config2_equals_grid_kernel(grid_frame, queue_renderer):
    """Config 2 (1200x800x500) through the queue kernel: the grid kernel's
    frame bit for bit, and the same number of world.hit calls."""
    img, segs = grid_frame
    got = queue_renderer.render(rt.final_camera(1.5), 1200, 800, 500, 50, SEED)
    assert queue_renderer.last_schedule()["persistent"] == 2
    assert queue_renderer.last_segments() == segs
    assert np.array_equal(got, img)


@pytest.mark.parametrize("G,g", [(8, 3), (3, 2)])
def test_queue_strip_equals_frame_rows(G, g, grid_frame, queue_renderer):
    """One rank's interleaved strip (chunked items: fewer tiles than 16 per
    resident block) equals those rows of the frame."""
    torch = pytest.importorskip("torch")
    img, _ = grid_frame
    W, H, S = 1200, 800, 500
    nrows = (H + G - 1) // G
    strip = torch.full((nrows, W, 3), -1.0, dtype=torch.float32, device="cuda:0")
    queue_renderer.render_rows(rt.final_camera(1.5), W, H, S, 50, SEED, g, G, nrows, strip.data_ptr(), 0)
    queue_renderer.synchronize()
    sch = queue_renderer.last_schedule()
    assert sch["persistent"] == 2 and sch["items_per_tile"] > 1, sch
    s = strip.cpu().numpy()
    nvalid = len(range(g, H, G))
    assert np.array_equal(s[:nvalid], img[g::G])
    assert not s[nvalid:].any()


def test_queue_progressive_passes(world, queue_renderer):
    W, H = 96, 64
    cam = rt.final_camera(W / H)
    want = O.fast_render(o_scene(world), o_cam(cam), W, H, 12, 50, SEED)
    queue_renderer.accum_reset(W, H)
    for s0, n in ((0, 5), (5, 1), (6, 6)):
        queue_renderer.render_pass(cam, W, H, s0, n)
    assert np.array_equal(queue_renderer.accum_resolve(), want)


def test_queue_watchdog_fault_is_reported(world, queue_renderer, monkeypatch):
    """a pass whose queue kernel's watchdog fired (injected here:
    RTMI_QUEUE_FAULT_INJECT=1 trips the idle watchdog at the first pass) left
    samples out; the fault is sticky until the next accumulator reset or
    whole render, so a resolve after that pass — and after further clean
    passes — fails with RT_EHIP, as does a render that faults itself.  A
    reset clears it and the same passes then resolve to the oracle's image."""
    W, H = 64, 40
    cam = rt.final_camera(W / H)
    queue_renderer.accum_reset(W, H)
    monkeypatch.setenv("RTMI_QUEUE_FAULT_INJECT", "1")
    queue_renderer.render_pass(cam, W, H, 0, 3)
    monkeypatch.delenv("RTMI_QUEUE_FAULT_INJECT")
    queue_renderer.render_pass(cam, W, H, 3, 3)
    for _ in range(2):
        with pytest.raises(rt.RTError, match="RT_EHIP"):
            queue_renderer.accum_resolve()
    queue_renderer.accum_reset(W, H)
    for s0 in (0, 3):
        queue_renderer.render_pass(cam, W, H, s0, 3)
    assert np.array_equal(queue_renderer.accum_resolve(), O.fast_render(o_scene(world), o_cam(cam), W, H, 6, 50, SEED))
    monkeypatch.setenv("RTMI_QUEUE_FAULT_INJECT", "1")
    with pytest.raises(rt.RTError, match="RT_EHIP"):
        queue_renderer.render(cam, W, H, 6, 50, SEED)
    monkeypatch.delenv("RTMI_QUEUE_FAULT_INJECT")
    assert np.array_equal(queue_renderer.render(cam, W, H, 6, 50, SEED),
                          O.fast_render(o_scene(world), o_cam(cam), W, H, 6, 50, SEED))


def test_queue_repeated_renders_are_identical(queue_renderer):
    """Scheduling differs run to run (waves race for rays); the image may not."""
    cam = rt.final_camera(1.5)
    a = queue_renderer.render(cam, 300, 200, 64, 50, SEED)
    for _ in range(3):
        assert np.array_equal(queue_renderer.render(cam, 300, 200, 64, 50, SEED), a)
