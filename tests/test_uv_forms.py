"""The fast mode's image-plane coordinates by reciprocals:
u = (i + r) * (1/(W-1)), v = (j + r) * (1/(H-1)) instead of main.cpp:278-279's
quotients.  The claim "<= 1 ulp from the quotient" is checked exhaustively by
the oracle (or_uv_forms): for the denominators of configs 1, 2 and 5 (both
axes), every numerator fl(i + r) the fast path can form — every column/row i
from 0 to W-1 (H-1), including the first and last, and every 24-bit jitter r.
CPU only (the kernels read the same reciprocal: tests/test_gpu_parity.py
pins the kernel to the oracle bit for bit)."""
import ctypes as C

import pytest

import oracle_py as O

CONFIGS = {"config1": (400, 225), "config2": (1200, 800), "config5": (3840, 2160)}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_reciprocal_coordinates_within_one_ulp_of_the_quotients(name):
    L = O.lib()
    L.or_uv_forms.argtypes = [C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.or_uv_forms.restype = C.c_int32
    for extent in CONFIGS[name]:
        D = extent - 1
        n, nd = C.c_int64(), C.c_int64()
        worst = L.or_uv_forms(D, C.byref(n), C.byref(nd))
        # 2^24 numerators below 1, then every float of [1, D + 1]
        assert n.value > (1 << 24) + (1 << 23) * (D.bit_length() - 1)
        assert worst <= 1, (name, extent, worst)
        # the forms do differ (6-55% of the numerators, by the one ulp):
        # the bound is not vacuous
        assert 0 < nd.value < n.value, (name, extent, nd.value, n.value)
