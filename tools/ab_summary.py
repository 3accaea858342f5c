"""Summarise a tools/gpu_ab_lib.sh output directory (<lib>_<rep>.json and
<lib>_s8_<rep>.json bench lines) into one table: kernel ms of config 2 and of
one rank's 1/8 strip per library and repetition.
    python tools/ab_summary.py gpurun_out/<tag>/ab "what was compared" > profiles/r03/<name>.txt"""
import glob
import json
import os
import re
import sys

d = sys.argv[1]
print(f"# {sys.argv[2] if len(sys.argv) > 2 else d}")
print("# kernel ms (HIP events, mean of 10 timed launches): config 2 frame | one rank's 1/8 strip")
rows = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    m = re.match(r"(.+?)(_s8)?_(\d+)\.json$", os.path.basename(f))
    if not m:
        continue
    try:
        ms = json.load(open(f))["roofline"]["kernel_ms"]
    except Exception:
        continue
    rows.setdefault(m.group(1), {}).setdefault("strip" if m.group(2) else "frame", []).append(ms)
for lib, v in rows.items():
    fr, st = v.get("frame", []), v.get("strip", [])
    print(f"{lib:12s} frame {' '.join(f'{x:.3f}' for x in fr):24s} strip8 {' '.join(f'{x:.3f}' for x in st)}")
