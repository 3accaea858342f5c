"""Analysis builds of librtmi (lib/librtmi_<name>.so) that a GPU script loads:
built here on the CPU with a stamp of the sources they were built from, and
checked against that stamp before a GPU run uses them, so a stale variant
(built before a kernel edit) is refused instead of measured (VERDICT r05
item 5).

    python tools/variants.py build NAME...   # make ... variant, then stamp
    python tools/variants.py check NAME...   # exit 1 unless built from the current sources
"""
import hashlib
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "csrc")
LIB = os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib")
# name -> (make target, flags)
VARIANTS = {
    "trace": ("variant", "-DRTMI_TRACE=1 -DRTMI_TRACE_PHASES=1"),  # per-wave timeline + phase clocks (tools/trace_run.py)
    "wavetrace": ("variant", "-DRTMI_TRACE=1"),  # per-wave timeline only (tools/gpu_trace_ab.sh)
    "nwph": ("nwvariant", "-DRTMI_NW_PHASES=1"),  # Next-Week phase clocks (tools/nw_phases.py)
    "w2": ("variant", "-DRTMI_BVH_WAVES=2"),  # 2-wave grid-kernel blocks (tools/gpu_small_blocks.sh)
    # compiler options for the device code (tools/gpu_variant_ab.sh)
    "f_prio": ("variant", "-mllvm -amdgpu-set-wave-priority"),
    "f_trk": ("variant", "-mllvm -amdgpu-use-amdgpu-trackers"),

}


def sources_digest():
    h = hashlib.sha1()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                   glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "Makefile")) +
                   glob.glob(os.path.join(REPO, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, REPO).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def stamp_path(name):
    return os.path.join(LIB, f"librtmi_{name}.so.stamp")


def build(name):
    target, flags = VARIANTS[name]
    subprocess.run(["make", "-C", CSRC, "-j8", target, f"NAME={name}", f"VFLAGS={flags}"], check=True)
    with open(stamp_path(name), "w") as f:
        f.write(f"{sources_digest()} {flags}\n")


def check(name):
    lib = os.path.join(LIB, f"librtmi_{name}.so")
    if not os.path.exists(lib) or not os.path.exists(stamp_path(name)):
        return f"{lib} not built: python tools/variants.py build {name} (on the CPU, before the GPU run)"
    built = open(stamp_path(name)).read().split()[0]
    if built != sources_digest():
        return f"{lib} is stale (built from other sources): python tools/variants.py build {name}"
    return None


def main():
    cmd, names = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        for n in names:
            build(n)
    elif cmd == "check":
        bad = [m for m in (check(n) for n in names) if m]
        for m in bad:
            print(m, file=sys.stderr)
        sys.exit(1 if bad else 0)
    else:
        sys.exit(__doc__)


if __name__ == "__main__":
    main()
