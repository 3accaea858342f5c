// rtmi_multi.hip — single-process multi-GPU render for the C++ drop-in path
// (SURVEY §8(e)).  The reference scales only over std::threads on contiguous
// pixel batches (main.cpp:318-338); here rows are interleaved over the GPUs
// (row j -> GPU j % G: per-row cost is uneven, contiguous strips would cap
// 8-GPU scaling at 6.08x, interleaving at 7.86x — SURVEY F8), each GPU
// renders its strip with the same kernel, and ONE RCCL gather moves the
// strips to GPU 0 over xGMI (per-GPU strip: ceil(H/G)*W*12 B; 1.44 MB at
// config 3).  Partition-invariant RNG keys make the image identical to the
// single-GPU render.
//
// bench.py's multi-GPU path is the one-process-per-GPU equivalent
// (torch.distributed over RCCL); this entry point serves C/C++ callers.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "rtmi_internal.h"

namespace rtmi {
hipStream_t ctx_stream(rt_ctx *ctx);  // rtmi_device.hip
}
using namespace rtmi;

namespace {
struct MultiState {
  std::vector<rt_ctx *> ctx;
  std::vector<float *> strip;
  std::vector<ncclComm_t> comm;
  float *recv = nullptr;
  ~MultiState() {
    for (auto c : comm)
      if (c) ncclCommDestroy(c);
    for (size_t g = 0; g < strip.size(); g++)
      if (strip[g]) { (void)hipSetDevice(int(g)); (void)hipFree(strip[g]); }
    if (recv) { (void)hipSetDevice(0); (void)hipFree(recv); }
    for (auto c : ctx) rt_ctx_destroy(c);
  }
};
}  // namespace

RTMI_EXPORT int rt_render_multi(const rt_scene *scene, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                                int32_t max_depth, uint64_t seed, int32_t n_gpus, float *sum) {
  if (!scene || !cam || !sum || W < 2 || H < 2 || spp < 1 || n_gpus < 0)
    return set_error(RT_EINVAL, "rt_render_multi: bad argument");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return set_error(RT_ENODEVICE, "no HIP device visible");
  const int G = n_gpus == 0 ? count : n_gpus;
  if (G > count) return set_error(RT_ENODEVICE, "asked for %d GPUs, %d visible", G, count);
  int prev = 0;
  (void)hipGetDevice(&prev);
  const int nrows = (H + G - 1) / G;
  const size_t strip_elems = size_t(nrows) * W * 3;
  int rc = RT_OK;
  {
    MultiState st;
    st.ctx.assign(G, nullptr);
    st.strip.assign(G, nullptr);
    for (int g = 0; g < G && rc == RT_OK; g++) {
      if ((rc = rt_ctx_create(g, &st.ctx[g]))) break;
      if ((rc = rt_ctx_set_scene(st.ctx[g], scene))) break;
      (void)hipSetDevice(g);
      if (hipMalloc(&st.strip[g], strip_elems * sizeof(float)) != hipSuccess)
        rc = set_error(RT_ENOMEM, "strip allocation on GPU %d", g);
    }
    if (rc == RT_OK) {
      (void)hipSetDevice(0);
      if (hipMalloc(&st.recv, strip_elems * G * sizeof(float)) != hipSuccess)
        rc = set_error(RT_ENOMEM, "gather buffer on GPU 0");
    }
    if (rc == RT_OK) {
      st.comm.assign(G, nullptr);
      std::vector<int> devs(G);
      for (int g = 0; g < G; g++) devs[g] = g;
      ncclResult_t r = ncclCommInitAll(st.comm.data(), G, devs.data());
      if (r != ncclSuccess) rc = set_error(RT_ERCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
    // render every strip (async, one stream per GPU)
    for (int g = 0; g < G && rc == RT_OK; g++)
      rc = rt_render_rows(st.ctx[g], cam, W, H, spp, max_depth, seed, g, G, nrows, st.strip[g], nullptr);
    // the single exchange step: gather strips to GPU 0
    if (rc == RT_OK) {
      std::vector<hipStream_t> streams(G);
      ncclResult_t r = ncclGroupStart();
      for (int g = 0; g < G && r == ncclSuccess; g++) {
        (void)hipSetDevice(g);
        hipStream_t s = rtmi::ctx_stream(st.ctx[g]);
        streams[g] = s;
        r = ncclGather(st.strip[g], g == 0 ? st.recv : nullptr, strip_elems, ncclFloat, 0, st.comm[g], s);
      }
      ncclResult_t r2 = ncclGroupEnd();
      if (r == ncclSuccess) r = r2;
      if (r != ncclSuccess) rc = set_error(RT_ERCCL, "ncclGather: %s", ncclGetErrorString(r));
      for (int g = 0; g < G && rc == RT_OK; g++) {
        (void)hipSetDevice(g);
        if (hipStreamSynchronize(streams[g]) != hipSuccess) rc = set_error(RT_EHIP, "sync GPU %d", g);
      }
      for (int g = 0; g < G && rc == RT_OK; g++) {
        ncclResult_t ae = ncclSuccess;
        ncclCommGetAsyncError(st.comm[g], &ae);
        if (ae != ncclSuccess) rc = set_error(RT_ERCCL, "RCCL async error on GPU %d: %s", g, ncclGetErrorString(ae));
      }
    }
    // un-permute: strip g row k is image row g + k*G
    if (rc == RT_OK) {
      std::vector<float> host(strip_elems * G);
      (void)hipSetDevice(0);
      if (hipMemcpy(host.data(), st.recv, host.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        rc = set_error(RT_EHIP, "gather buffer copy");
      for (int g = 0; g < G && rc == RT_OK; g++)
        for (int k = 0; k < nrows; k++) {
          const int j = g + k * G;
          if (j >= H) break;
          std::memcpy(sum + size_t(j) * W * 3, host.data() + (size_t(g) * nrows + k) * W * 3, size_t(W) * 3 * sizeof(float));
        }
    }
  }
  (void)hipSetDevice(prev);
  return rc;
}
