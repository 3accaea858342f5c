import os, sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import a_dive_into_ray_tracing_amd as rt, oracle_py as O, ctypes as C
w = rt.random_scene(); r = rt.Renderer(w, 0); r.set_accel("grid")
print("grid info", r.grid_info())
cam = rt.final_camera(96/64)
got = r.render(cam, 96, 64, 8, 50, 1984)
oc = O.OrCamera(); C.memmove(C.byref(oc), C.byref(cam), C.sizeof(oc))
want = O.fast_render(O.Scene(w.center_radius, w.mat_kind, w.mat_params), oc, 96, 64, 8, 50, 1984)
print("direct bit-exact:", np.array_equal(got, want))
