"""rt_multi_* at G > 1 on one GPU through the mock gather.

RTMI_MULTI_MOCK=1 maps logical device g onto physical device g % visible,
each with its own context and stream, and replaces ncclCommInitAll /
ncclGather with a peer copy of each strip into device 0's receive buffer
after that strip's end event (csrc/rtmi_multi.hip).  Everything else is the
product's multi-device code: per-device streams and events, the cross-device
waits before the gather, the drains after a partial failure, progressive
passes and rt_unpermute_rows.  RCCL itself is the only piece these tests do
not reach; it runs on the driver's 8-GPU node.

The partition being replaced is the reference's 16-thread contiguous batch
split (rt_in_one_weekend/main.cpp:318-338); rows are interleaved here (row j
on device j % G), and per-(pixel, sample) RNG keys make every G give the
single-device bits.
"""
import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt

pytestmark = pytest.mark.gpu
SEED = 1984


@pytest.fixture(scope="module")
def world():
    return rt.random_scene()


@pytest.fixture(scope="module")
def single(world):
    r = rt.Renderer(world, 0)
    yield r
    r.close()


@pytest.fixture
def mock(monkeypatch):
    monkeypatch.setenv("RTMI_MULTI_MOCK", "1")
    monkeypatch.delenv("RTMI_MULTI_MOCK_FAIL", raising=False)
    return monkeypatch


@pytest.mark.parametrize("G", [2, 3, 8])
def test_mock_multi_render_equals_render(G, world, single, mock):
    """rt_multi_render at G logical devices == rt_render, bit for bit, for
    an H that G does not divide (padded strips), twice on the same set; the
    timing reports G strips and a gather."""
    W, H, S = 40, 30, 6
    cam = rt.final_camera(W / H)
    want = single.render(cam, W, H, S, 50, SEED)
    m = rt.MultiRenderer(world, n_gpus=G)
    try:
        assert m.n_gpus == G
        for _ in range(2):
            assert np.array_equal(m.render(cam, W, H, S, 50, SEED), want)
        strip_ms, gather_ms = m.last_timing()
        assert len(strip_ms) == G and all(t > 0 for t in strip_ms) and gather_ms >= 0
        # a larger image on the same set: strips and the gather buffer grow
        W2, H2 = 64, 45
        cam2 = rt.final_camera(W2 / H2)
        assert np.array_equal(m.render(cam2, W2, H2, 3, 50, SEED), single.render(cam2, W2, H2, 3, 50, SEED))
    finally:
        m.close()


@pytest.mark.parametrize("G", [2, 3, 8])
def test_mock_multi_progressive_passes_resolve_to_render(G, world, single, mock):
    W, H = 36, 20
    cam = rt.final_camera(W / H)
    want = single.render(cam, W, H, 7, 50, SEED)
    m = rt.MultiRenderer(world, n_gpus=G)
    try:
        m.accum_reset(W, H)
        for s0, n in ((0, 2), (2, 1), (3, 4)):
            m.render_pass(cam, s0, n)
        assert np.array_equal(m.accum_resolve(), want)
        assert len(m.last_timing()[0]) == G
    finally:
        m.close()


def test_mock_multi_pass_failing_on_device_2_of_3_invalidates(world, single, mock):
    """A pass that fails on logical device 2 of 3 after devices 0 and 1 have
    enqueued theirs (the drain's case): the error is returned
    with the earlier devices drained, rt_multi_accum_resolve and further
    passes refuse until rt_multi_accum_reset, and a reset set resolves to
    the one-render bits."""
    W, H = 24, 16
    cam = rt.final_camera(W / H)
    m = rt.MultiRenderer(world, n_gpus=3)
    try:
        m.accum_reset(W, H)
        m.render_pass(cam, 0, 2)
        mock.setenv("RTMI_MULTI_MOCK_FAIL", "2")
        with pytest.raises(RuntimeError, match="injected failure on logical device 2"):
            m.render_pass(cam, 2, 2)
        mock.delenv("RTMI_MULTI_MOCK_FAIL")
        with pytest.raises(RuntimeError, match="no accumulator"):
            m.accum_resolve()
        with pytest.raises(RuntimeError, match="no accumulator"):
            m.render_pass(cam, 2, 2)
        m.accum_reset(W, H)
        m.render_pass(cam, 0, 2)
        m.render_pass(cam, 2, 2)
        assert np.array_equal(m.accum_resolve(), single.render(cam, W, H, 4, 50, SEED))
    finally:
        m.close()


@pytest.mark.parametrize("fail_on", [1, 7])
def test_mock_multi_render_failing_on_a_later_device_recovers(fail_on, world, single, mock):
    """rt_multi_render failing on logical device g > 0 (devices 0..g-1
    already rendering their strips) returns the error after draining them;
    the same set then renders the single-device bits."""
    W, H, S = 32, 24, 4
    cam = rt.final_camera(W / H)
    m = rt.MultiRenderer(world, n_gpus=8)
    try:
        mock.setenv("RTMI_MULTI_MOCK_FAIL", str(fail_on))
        with pytest.raises(RuntimeError, match=f"injected failure on logical device {fail_on}"):
            m.render(cam, W, H, S, 50, SEED)
        mock.delenv("RTMI_MULTI_MOCK_FAIL")
        assert np.array_equal(m.render(cam, W, H, S, 50, SEED), single.render(cam, W, H, S, 50, SEED))
    finally:
        m.close()


def test_mock_multi_resolve_failing_keeps_accumulators(world, single, mock):
    """A resolve that fails on logical device 1 of 2 leaves the accumulators
    valid (nothing was added to them): the next resolve returns the bits."""
    W, H = 20, 12
    cam = rt.final_camera(W / H)
    m = rt.MultiRenderer(world, n_gpus=2)
    try:
        m.accum_reset(W, H)
        m.render_pass(cam, 0, 3)
        mock.setenv("RTMI_MULTI_MOCK_FAIL", "1")
        with pytest.raises(RuntimeError, match="injected failure"):
            m.accum_resolve()
        mock.delenv("RTMI_MULTI_MOCK_FAIL")
        assert np.array_equal(m.accum_resolve(), single.render(cam, W, H, 3, 50, SEED))
    finally:
        m.close()


def test_without_mock_more_devices_than_visible_is_refused(world):
    import ctypes as C
    import os
    assert not os.environ.get("RTMI_MULTI_MOCK")
    n = C.c_int32()
    L = rt.load()
    assert L.rt_device_count(C.byref(n)) == 0
    h = C.c_void_p()
    sc = world.c_struct()
    assert L.rt_multi_create(C.byref(sc), n.value + 1, C.byref(h)) == -3 and not h.value  # RT_ENODEVICE
