"""Debug: where the GPU Next-Week image differs from the oracle (scene argv[1])."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import a_dive_into_ray_tracing_amd.nextweek as nw  # noqa: E402
import oracle_py as O  # noqa: E402

which = int(sys.argv[1])
W, H, spp = 29, 23, int(sys.argv[2]) if len(sys.argv) > 2 else 1
s, cam = nw.preset(which, image=None, aspect=W / H)
r = nw.NwRenderer(s)
got = r.render(cam, W, H, spp, 50, 1984)
segs = r.last_segments()
want, wsegs = O.nw_render(s.flat(), cam, W, H, spp, 50, 1984)
d = np.abs(got - want).max(axis=2)
print("segments", segs, wsegs, "differing pixels", int((d > 0).sum()), "of", W * H)
for j, i in list(zip(*np.nonzero(d)))[:8]:
    print(j, i, got[j, i], want[j, i])

# first differing pixel: which of its samples differ, and where the paths part
for j, i in list(zip(*np.nonzero(d)))[:1]:
    for smp in range(spp):
        g, gk = r.debug_trace(cam, W, H, int(i), int(j), smp)
        w, wk = O.nw_trace(s.flat(), cam, W, H, 50, 1984, int(i), int(j), smp)
        if g.shape == w.shape and np.array_equal(g, w) and np.array_equal(gk, wk):
            continue
        print("pixel", j, i, "sample", smp, "segments", len(g), len(w))
        for q in range(min(len(g), len(w))):
            same = np.array_equal(g[q], w[q]) and np.array_equal(gk[q], wk[q])
            print(q, "same" if same else "DIFF", "gpu", g[q].tolist(), gk[q].tolist(), "oracle", w[q].tolist(), wk[q].tolist())
            if not same:
                break
r.close()
