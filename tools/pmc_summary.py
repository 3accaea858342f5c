"""Summarise rocprofv3 PMC csvs of the render kernels: per-dispatch means,
grouped by kernel (render and finalize kernels); "renders" leaves out dispatches
below a quarter of the largest (the cost probe).  usage: pmc_summary.py DIR"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc*/*_counter_collection.csv")):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if any(n in k for n in ("render_kernel", "render_persistent", "render_queue", "render_resident", "finalize_kernel")):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = k.split("(")[0]
    for (dsp, c), v in per.items():
        vals[names[dsp]][c].append(v)
for k in sorted(vals):
    print(k)
    for c in sorted(vals[k]):
        v = vals[k][c]
        # the renders proper: a one-shot render's cost probe (a few spp, the
        # same kernel) is a dispatch far smaller than the rest
        big = [x for x in v if x >= 0.25 * max(v)] if max(v) > 0 else v
        print(f"  {c:32s} mean {sum(v)/len(v):.4g}  (n={len(v)})  renders {sum(big)/len(big):.4g}  (n={len(big)})")
