"""Print the register / scratch / LDS budget of the render kernels in a built
library (no GPU needed): python tools/kernel_resources.py [lib.so] [filter].

Reads the gfx950 code objects' AMDGPU metadata the same way
tests/test_kernel_resources.py does."""
import os
import sys
import tempfile
import pathlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import test_kernel_resources as K  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else K.LIB
    pat = sys.argv[2] if len(sys.argv) > 2 else "render_"
    K.LIB = lib
    with tempfile.TemporaryDirectory() as d:
        meta = K.kernel_metadata(pathlib.Path(d))
    for name in sorted(meta):
        if pat in name:
            m = meta[name]
            print(f"{name:60s} vgpr {m.get('vgpr_count')} scratch {m.get('private_segment_fixed_size')} "
                  f"spill {m.get('vgpr_spill_count', 0)} lds {m.get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
