"""tools/variants.py: an analysis build is usable on the
GPU box only while it was built from the current sources — its stamp holds
the digest of csrc/, include/ and the Makefile at build time, and the check
refuses a library that is missing, unstamped or stamped from other sources.
CPU only: the stamps are checked against a copy of the tree, no GPU needed."""
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_variant_check_refuses_missing_and_stale(tmp_path, monkeypatch):
    root = tmp_path / "repo"
    for d in ("a_dive_into_ray_tracing_amd/csrc", "include", "tools"):
        shutil.copytree(os.path.join(REPO, d), root / d, ignore=shutil.ignore_patterns("build", "*.o"))
    (root / "a_dive_into_ray_tracing_amd" / "lib").mkdir(parents=True)
    sys.path.insert(0, str(root / "tools"))
    try:
        import importlib

        import variants
        importlib.reload(variants)  # (bound to the copy's paths)
        assert "not built" in variants.check("trace")
        lib = root / "a_dive_into_ray_tracing_amd" / "lib" / "librtmi_trace.so"
        lib.write_bytes(b"\x7fELF stand-in")
        assert "not built" in variants.check("trace")  # no stamp
        with open(variants.stamp_path("trace"), "w") as f:
            f.write(variants.sources_digest() + " -DRTMI_TRACE=1\n")
        assert variants.check("trace") is None  # built from these sources
        src = root / "a_dive_into_ray_tracing_amd" / "csrc" / "rtmi_path.h"
        src.write_text(src.read_text() + "\n// an edit after the build\n")
        assert "stale" in variants.check("trace")
    finally:
        sys.path.remove(str(root / "tools"))
        sys.modules.pop("variants", None)
