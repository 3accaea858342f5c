"""Summarise rocprofv3 PMC csvs of the render kernel: per-dispatch sums."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "render_kernel" in r["Kernel_Name"] or "render_persistent" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c in sorted(vals):
    v = vals[c]
    print(f"{c:32s} mean {sum(v)/len(v):.4g}  (n={len(v)})")
