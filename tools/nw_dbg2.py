import os, sys
import numpy as np
REPO = os.getcwd()
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import a_dive_into_ray_tracing_amd.nextweek as nw
import oracle_py as O
W, H = 29, 23
s, cam = nw.preset(6, image=None, aspect=W / H)
r = nw.NwRenderer(s)
g, gk = r.debug_trace(cam, W, H, 22, 3, 0)
w, wk = O.nw_trace(s.flat(), cam, W, H, 50, 1984, 22, 3, 0)
np.set_printoptions(precision=9, suppress=False, linewidth=200)
print("GPU"); print(np.column_stack([g, gk[:, :1]]))
print("ORACLE"); print(np.column_stack([w, wk]))
print("info", r.info())
