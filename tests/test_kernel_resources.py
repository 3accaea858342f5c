"""The built library's render kernels keep the register budget DESIGN.md
§4.5/§8 rests on (no GPU needed): the one-layer grid kernel that renders the
final scene, render_kernel<8, true, 3>, and its cost probe <8, false, 3> use
at most 64 VGPRs (8 waves per SIMD) and no private segment (no spills), and
their static LDS leaves the grid's record slots room for 8 blocks per CU.

The code objects are read from the library's .hip_fatbin section (clang
offload bundles, one per linked HIP object) and their AMDGPU metadata notes
printed by llvm-readelf."""
import os
import re
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def gfx950_code_objects(fatbin):
    """Every gfx950 entry of every offload bundle in the section."""
    out, pos = [], fatbin.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", fatbin, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fatbin, p)
            triple = fatbin[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith("gfx950"):
                out.append(fatbin[pos + off:pos + off + size])
        pos = fatbin.find(MAGIC, pos + 1)
    return out


def kernel_metadata(tmp_path):
    """{kernel symbol: {field: value}} from the notes of all code objects."""
    sec = tmp_path / "fat.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", LIB, str(tmp_path / "copy.so")],
                   check=True, capture_output=True)
    meta = {}
    for i, co in enumerate(gfx950_code_objects(sec.read_bytes())):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(co)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(f)], check=True, capture_output=True,
                               text=True).stdout
        # one block per kernel in the amdhsa.kernels list
        for block in re.split(r"\n\s+- \.", notes):
            m = re.search(r"\.symbol:\s+(\S+)", block)
            if not m:
                continue
            fields = dict(re.findall(r"\.(vgpr_count|private_segment_fixed_size|group_segment_fixed_size"
                                     r"|vgpr_spill_count|sgpr_spill_count|sgpr_count):\s+(\d+)", "." + block))
            meta[m.group(1)] = {k: int(v) for k, v in fields.items()}
    return meta


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf")),
                    reason="needs the built library and ROCm's llvm tools")
def test_frame_kernel_register_budget(tmp_path):
    meta = kernel_metadata(tmp_path)
    for chunked in ("1", "0"):
        name = [k for k in meta if f"render_kernelILi8ELb{chunked}ELi3E" in k]
        assert len(name) == 1, sorted(meta)[:20]
        m = meta[name[0]]
        assert m["vgpr_count"] <= 64, (name[0], m)  # 8 waves per SIMD
        assert m["private_segment_fixed_size"] == 0, (name[0], m)  # no scratch: no spills
        assert m.get("vgpr_spill_count", 0) == 0, (name[0], m)
        # static LDS (camera, block counters, grid descriptor): the 20 KB a block
        # may use at 8 blocks per CU minus the record slots and sums (§4.5)
        assert m["group_segment_fixed_size"] <= 256, (name[0], m)


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf")),
                    reason="needs the built library and ROCm's llvm tools")
def test_product_library_holds_no_experimental_kernel(tmp_path):
    """the kernels that measured slower than the grid
    kernel are not in librtmi.so (the resident kernel is in the experimental
    build only, the queue kernel retired); the product's render kernels are
    all there."""
    meta = kernel_metadata(tmp_path)
    assert not [k for k in meta if "render_queue" in k or "render_resident" in k]
    assert [k for k in meta if "render_kernelILi8ELb1ELi3E" in k]
