"""profiles/pmc_valu.json from tools/profile.sh's PMC passes: per-launch
VALU counters of the timed render kernel (config 2, grid), which bench.py
reports beside the algorithmic roofline as roofline.pmc.
usage: pmc_valu_json.py PROFILE_DIR KERNEL_MS SOURCE_NOTE [KERNEL] > profiles/pmc_valu.json
(KERNEL default: the one-layer grid instantiation render_kernel<8, true, 3>).
The record carries the kernel's symbol fragment and the sha1 of its gfx950 code
in the library these passes ran (RTMI_LIBRARY or lib/librtmi.so): bench.py
quotes it only while the timed kernel hashes the same."""
import collections
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from a_dive_into_ray_tracing_amd import codeobj  # noqa: E402


def symbol_of(name):
    """'rtmi::render_kernel<8, true, 3>' -> 'render_kernelILi8ELb1ELi3E' (Itanium mangling of the arguments)."""
    base, args = re.match(r"rtmi::(\w+)<(.*)>", name).groups()
    parts = []
    for a in (x.strip() for x in args.split(",")):
        parts.append({"true": "Lb1E", "false": "Lb0E"}.get(a, f"Li{a}E"))
    return base + "I" + "".join(parts)

root, kernel_ms, note = sys.argv[1], float(sys.argv[2]), sys.argv[3]
want = sys.argv[4] if len(sys.argv) > 4 else "rtmi::render_kernel<8, true, 3>"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].split("(")[0].replace("void ", "") == want:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, c), v in per.items():
        vals[c].append(v)
m = {c: sum(v) / len(v) for c, v in vals.items()}
lib = os.environ.get("RTMI_LIBRARY") or os.path.join(REPO, "a_dive_into_ray_tracing_amd", "lib", "librtmi.so")
sym = symbol_of(want)
out = {
    "source": note,
    "kernel": want,
    "symbol": sym,
    "code_sha1": codeobj.kernel_sha1(lib, sym)[1],
    "code_sha1_note": ("sha1 of the kernel's gfx950 machine code in librtmi.so (a_dive_into_ray_tracing_amd/codeobj.py); "
                       "bench.py quotes these counts only while the timed kernel's code hashes the same"),
    "kernel_ms_of_that_tree": kernel_ms,
    "per_launch": {c: m[c] for c in sorted(m)},
    "executed_fp32_flop_per_launch": 64 * m["SQ_INSTS_VALU_FLOPS_FP32"],
    "lane_utilisation": m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]),
    "wait_fraction": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"],
    "definitions": {
        "executed_fp32_flop_per_launch": "64 x SQ_INSTS_VALU_FLOPS_FP32 (the counter counts per 64 lanes; x64 reproduced the "
                                         "brute-force kernel's algorithmic FLOP, DESIGN.md section 5)",
        "lane_utilisation": "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)",
        "wait_fraction": "SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES",
        "valu_issue_busy (bench.py)": "SQ_INSTS_VALU x 2 cycles (one wave64 FP32 op per 2 cycles per SIMD on gfx950) / "
                                      "(1024 SIMDs x 2.4 GHz x kernel time); a lower bound: 64-bit and transcendental "
                                      "ops issue for longer",
    },
}
print(json.dumps(out, indent=1))
