"""Per-launch GPU time of the render kernel from a rocprofv3 kernel trace
(<prefix>_kernel_trace.csv): launch count, mean start-to-end duration, and the
union of the launches' intervals / count — the figure bench.py reports as
roofline.kernel_ms when consecutive steps' launches overlap on two streams
(--pipeline 2).  Only launches of the most common grid size count (the
timed renders; cost probes and side launches have other grids).
usage: trace_busy.py <kernel_trace.csv> [kernel-name substring]"""
import collections
import csv
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
if not rows:
    sys.exit(f"no {name} launches in {path}")
grid = collections.Counter(r["Grid_Size_X"] for r in rows).most_common(1)[0][0]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if r["Grid_Size_X"] == grid)
busy, (s0, e0) = 0, iv[0]
for s, e in iv[1:]:
    if s > e0:
        busy += e0 - s0
        s0, e0 = s, e
    else:
        e0 = max(e0, e)
busy += e0 - s0
mean = sum(e - s for s, e in iv) / len(iv)
queues = sorted({r["Queue_Id"] for r in rows if r["Grid_Size_X"] == grid})
print(f"{name} (grid {grid}): {len(iv)} launches on queues {','.join(queues)}; mean duration {mean / 1e6:.3f} ms; "
      f"busy (union of intervals) per launch {busy / len(iv) / 1e6:.3f} ms")
