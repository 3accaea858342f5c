"""Analysis: K back-to-back renders of one workload on one stream (one
context) against the same renders alternating over two contexts on two
streams (consecutive launches may overlap: the next render's blocks fill the
CUs as the previous one's last blocks drain).  Prints wall ms per render.
usage: overlap_probe.py [rows_of_N (1 = whole frame)] [K]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import a_dive_into_ray_tracing_amd as rt  # noqa: E402
from a_dive_into_ray_tracing_amd import dist as rdist  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W, H, S = 1200, 800, 500
world = rt.random_scene()
cam = rt.final_camera(W / H)
row0, step, nrows = rdist.strip_rows(H, 0, N)
dev = torch.device("cuda", 0)
bufs = [torch.empty((nrows, W, 3), dtype=torch.float32, device=dev) for _ in range(2)]
rs = [rt.Renderer(world, 0) for _ in range(2)]
if os.environ.get("OV_CTX_STREAMS") == "1":
    class _Z:  # each context's own stream (rt_render_rows with stream 0)
        cuda_stream = 0
    ss = [_Z(), _Z()]
elif os.environ.get("OV_HIP_STREAMS", "1") == "1":
    # streams made by the HIP runtime directly (torch's pool put both on one hardware queue)
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    torch.cuda.synchronize()
    class _S:
        def __init__(self, prio):
            h = C.c_void_p()
            if os.environ.get("OV_CUMASK") == "1":  # a CU-masked stream (all CUs): its own hardware queue?
                mask = (C.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
                assert hip.hipExtStreamCreateWithCUMask(C.byref(h), 8, mask) == 0
            else:
                assert hip.hipStreamCreateWithPriority(C.byref(h), 1, prio) == 0
            self.cuda_stream = h.value
    # OV_PRIO="a,b": the two streams' priorities (HIP: lower is higher)
    pr = [int(x) for x in os.environ.get("OV_PRIO", "0,0").split(",")]
    ss = [_S(pr[0]), _S(pr[1])]
else:
    ss = [torch.cuda.Stream(dev) for _ in range(2)]
for r in rs:
    r.set_accel("grid")


def run(nctx):
    for k in range(4):  # warm-up: cost maps of this layout in both contexts
        i = k % 2
        rs[i].render_rows(cam, W, H, S, 50, 1984, row0, step, nrows, bufs[i].data_ptr(), ss[i].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        i = k % nctx
        rs[i].render_rows(cam, W, H, S, 50, 1984, row0, step, nrows, bufs[i].data_ptr(), ss[i].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for rep in range(2):
    one = run(1)
    two = run(2)
    print(f"1/{N} of config 2, {K} renders: one stream {one:.3f} ms/render, two streams {two:.3f} ms/render "
          f"({100 * (two / one - 1):+.1f}%)", flush=True)
assert torch.equal(bufs[0], bufs[1])
print("images identical")
for r in rs:
    r.close()
if os.environ.get("OV_CTX_STREAMS") != "1" and os.environ.get("OV_HIP_STREAMS", "1") == "1":
    for x in ss:
        assert hip.hipStreamDestroy(C.c_void_p(x.cuda_stream)) == 0
