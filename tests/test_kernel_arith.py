"""Host checks of integer identities the kernels rely on (no GPU needed).

render_kernel decodes a job q into (sample, pixel) and a pixel into (row,
column) by q / d = umulhi(2q, ceil(2^31 / d)) (rtmi_device.hip, camera_ray /
adopt): exact for every tile size d in 1..64 and every job index the host
allows (q < 64 * 65535 < 2^22, rtmi_device.hip's chunk clamp)."""
import numpy as np


def test_job_division_by_reciprocal_multiply_is_exact():
    q = np.arange(1 << 22, dtype=np.uint64)
    for d in range(1, 65):
        m = np.uint64(0x7FFFFFFF // d + 1)
        assert np.array_equal(((q << np.uint64(1)) * m) >> np.uint64(32), q // np.uint64(d)), d
