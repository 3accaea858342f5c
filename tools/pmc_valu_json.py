"""profiles/pmc_valu.json from tools/profile.sh's PMC passes: per-launch
VALU counters of the timed render kernel (config 2, grid), which bench.py
reports beside the algorithmic roofline as roofline.pmc.
usage: pmc_valu_json.py PROFILE_DIR KERNEL_MS SOURCE_NOTE [KERNEL] > profiles/pmc_valu.json
(KERNEL default: the one-layer grid instantiation render_kernel<8, true, 3>)"""
import collections
import csv
import glob
import json
import sys

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
out = {
    "source": note,
    "kernel": want,
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
