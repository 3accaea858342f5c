"""The resident grid kernel (RT_KERNEL_RESIDENT), measured
slower than the grid kernel, lives only in the experimental build
(lib/librtmi_experimental.so, `make -C a_dive_into_ray_tracing_amd/csrc
experimental`); the queue kernel (RT_KERNEL_QUEUE, §4.6) was retired.  The
product library runs the automatic choice for both kinds (same image); the
experimental build's own suite (tests/experimental/exp_gpu_resident.py:
bit-exact against the oracle and the grid kernel) runs in ONE child process,
since a process loads one library."""
import os
import subprocess
import sys

import numpy as np
import pytest

import a_dive_into_ray_tracing_amd as rt

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP_LIB = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi_experimental.so")


@pytest.mark.parametrize("kind", ["queue", "resident"])
def test_product_runs_the_automatic_kernel_for_experimental_kinds(kind):
    w = rt.random_scene()
    cam = rt.final_camera(1.5)
    r = rt.Renderer(w, 0)
    try:
        want = r.render(cam, 120, 80, 16, 50, 1984)
        r.set_kernel(kind)
        got = r.render(cam, 120, 80, 16, 50, 1984)
        assert r.last_schedule()["persistent"] == 0  # the grid kernel ran
    finally:
        r.close()
    assert np.array_equal(got, want)


@pytest.mark.skipif(not os.path.exists(EXP_LIB), reason="experimental build absent (make ... experimental)")
def test_experimental_build_suite():
    env = dict(os.environ, RTMI_LIBRARY=EXP_LIB)
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    p = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-v", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "experimental", "exp_gpu_resident.py")],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    with open(os.path.join(out, "experimental_suite.log"), "w") as f:
        f.write(p.stdout + p.stderr)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
