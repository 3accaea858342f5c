"""The fast-mode restatement (the kernel's numerics contract) against the
reference semantics, on the CPU.

Fast mode is the reference algorithm in float with a counter-based RNG and a
float-robustness ray offset.  Its per-sample paths cannot
match the double/glibc reference path-for-path, so it is held to
the reference statistically: same mean path length (world.hit calls per
sample) and same mean radiance as the ref-mode restatement, which is itself
bit-exact against the reference (test_oracle_golden.py)."""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

W, H, S = 120, 80, 48


@pytest.fixture(scope="module")
def renders():
    sc, g = O.final_scene()
    cam = O.final_camera(W / H)
    ref, _ = O.ref_worker(sc, cam, W, H, S, 50, 0, W * H, g)
    ref_segs = O.lib().or_ref_last_segments()
    fast = O.fast_render(sc, cam, W, H, S, 50, 1984)
    fast_segs = O.fast_segments(sc, cam, W, H, S, 50, 1984)
    return sc, cam, ref.reshape(H, W, 3) / S, ref_segs, fast / S, fast_segs


def test_path_length_matches_reference(renders):
    """Without the ray offset, float acne inflates this by ~8%."""
    _, _, _, ref_segs, _, fast_segs = renders
    n = W * H * S
    assert abs(fast_segs / n - ref_segs / n) < 0.01 * ref_segs / n, (fast_segs / n, ref_segs / n)


def test_mean_radiance_matches_reference(renders):
    _, _, ref, _, fast, _ = renders
    # per-pixel means of S samples; the image mean's MC std is ~1e-3 here
    for c in range(3):
        assert abs(fast[..., c].mean() - ref[..., c].mean()) < 4e-3
    # 8x8-pixel tile means agree to within their own noise
    tr = ref.reshape(10, 8, 15, 8, 3).mean(axis=(1, 3))
    tf = fast.reshape(10, 8, 15, 8, 3).mean(axis=(1, 3))
    assert np.abs(tr - tf).mean() < 0.02


def test_fast_mode_partition_invariant(renders):
    sc, cam, _, _, fast, _ = renders
    G = 3
    nrows = (H + G - 1) // G
    for g in range(G):
        strip = O.fast_render(sc, cam, W, H, S, 50, 1984, row0=g, row_step=G, nrows=nrows) / S
        for k in range(nrows):
            j = g + k * G
            if j < H:
                assert np.array_equal(strip[k], fast[j])
            else:
                assert not strip[k].any()


def test_fast_rng_streams_distinct():
    a = np.zeros(8, np.uint64)
    b = np.zeros(8, np.uint64)
    O.lib().or_fast_rng(1984, 5, 0, 8, a.ctypes.data_as(C.POINTER(C.c_uint64)))
    O.lib().or_fast_rng(1984, 5, 1, 8, b.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert not np.array_equal(a, b)
    O.lib().or_fast_rng(1984, 6, 0, 8, b.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert not np.array_equal(a, b)
