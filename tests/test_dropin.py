"""The drop-in: rt_in_one_weekend's own parallel_render() with its thread
block replaced by rtmi::render (include/rtmi.hpp), compiled from the
reference sources by oracle/Makefile into oracle/_ref/dropin_demo.

CPU: the adapter compiles against the reference's headers and links
librtmi.so; without a GPU it fails loudly (no CPU fallback).
GPU: its PPM equals our own driver's image at the same seed, pixel for pixel.
"""
import os
import subprocess

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(REPO, "oracle", "_ref", "dropin_demo")
HAVE_REF = os.path.isdir("/root/reference/rt_in_one_weekend")


def test_adapter_compiles_against_reference_headers():
    if not HAVE_REF:
        pytest.skip("reference sources not present (GPU box)")
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True, capture_output=True)
    assert os.access(DEMO, os.X_OK)


def test_dropin_without_gpu_fails_loudly():
    if not os.path.exists(DEMO):
        pytest.skip("drop-in demo not built")
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([DEMO, "24", "2"], capture_output=True, text=True)
    assert r.returncode != 0 and "no HIP device" in r.stderr


def _p3(text):
    tok = text.split()
    assert tok[0] == "P3"
    w, h = int(tok[1]), int(tok[2])
    return np.array(tok[4:], np.int64).reshape(h, w, 3)


@pytest.mark.gpu
def test_dropin_image_equals_rt_render():
    if not os.path.exists(DEMO):
        pytest.skip("drop-in demo not built (needs the reference sources at build time)")
    W, S = 120, 16
    H = int(W / 1.5)
    r = subprocess.run([DEMO, str(W), str(S)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    theirs = _p3(r.stdout)
    ours = rt.quantize(rt.render(W, H, S, 50, rt.random_scene(), rt.final_camera(W / H), seed=1984), S)
    assert np.array_equal(theirs, ours.astype(np.int64))
