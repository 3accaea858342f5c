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
// rt_multi keeps everything a render needs across calls — one context per
// device with the scene resident, the strips, the gather buffer and the RCCL
// communicator (ncclCommInitAll once) — and times each render per device
// (HIP events around each device's strip) and the gather alone (device 0's
// stream waits for every strip before the gather's start event), so a loss
// of scaling can be attributed to a slow strip or to the exchange.
//
// bench.py's multi-GPU path is the one-process-per-GPU equivalent
// (torch.distributed over RCCL); this entry point serves C/C++ callers.
//
// Mock gather (analysis and tests only): with
// RTMI_MULTI_MOCK=1 in the environment at rt_multi_create, logical device g
// runs on physical device g % visible (each logical device its own context and
// stream, so G logical devices can share one GPU) and the gather is a
// peer copy of each strip into device 0's receive buffer on device 0's stream
// after that strip's end event, in place of ncclCommInitAll / ncclGather.
// Everything else is the product's code: streams, events, drains, progressive
// passes, rt_unpermute_rows.  With the mock, RTMI_MULTI_MOCK_FAIL=g (read per
// call) makes rt_multi_render / _render_pass / _accum_resolve fail on logical
// device g after devices 0..g-1 have enqueued their work: the partial-failure
// path the drains exist for.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "rtmi_internal.h"

namespace rtmi {
hipStream_t ctx_stream(rt_ctx *ctx);  // rtmi_device.hip
}
using namespace rtmi;

struct rt_multi {
  int G = 0;
  std::vector<rt_ctx *> ctx;
  std::vector<float *> strip;
  size_t strip_cap = 0;  // elements per strip
  float *recv = nullptr;
  size_t recv_cap = 0;  // elements
  std::vector<ncclComm_t> comm;
  std::vector<hipEvent_t> ev_begin, ev_end;  // per device, on its context's stream
  hipEvent_t gather_begin = nullptr, gather_end = nullptr;  // device 0
  std::vector<float> host;
  std::vector<float> strip_ms;
  float gather_ms = -1.0f;
  int32_t pass_W = 0, pass_H = 0, pass_nrows = 0;  // progressive accumulators (0: none)
  int visible = 1;    // physical devices
  bool mock = false;  // RTMI_MULTI_MOCK: logical devices over the visible ones, copy gather
  int dev(int g) const { return mock ? g % visible : g; }  // logical -> physical device
};

namespace {
void destroy(rt_multi *m) {
  if (!m) return;
  for (int g = 0; g < int(m->ctx.size()); g++)
    if (m->ctx[g]) { (void)hipSetDevice(m->dev(g)); (void)rt_ctx_synchronize(m->ctx[g]); }
  for (auto c : m->comm)
    if (c) ncclCommDestroy(c);
  for (size_t g = 0; g < m->strip.size(); g++) {
    (void)hipSetDevice(m->dev(int(g)));
    if (m->strip[g]) (void)hipFree(m->strip[g]);
    if (g < m->ev_begin.size() && m->ev_begin[g]) (void)hipEventDestroy(m->ev_begin[g]);
    if (g < m->ev_end.size() && m->ev_end[g]) (void)hipEventDestroy(m->ev_end[g]);
  }
  (void)hipSetDevice(m->dev(0));
  if (m->recv) (void)hipFree(m->recv);
  if (m->gather_begin) (void)hipEventDestroy(m->gather_begin);
  if (m->gather_end) (void)hipEventDestroy(m->gather_end);
  for (auto c : m->ctx) rt_ctx_destroy(c);
  delete m;
}

// After a failure part-way through a multi-device call, some devices' streams
// may still hold enqueued work (strips, passes, a gather) that reads or writes
// this object's buffers and records its events: wait for all of it before
// returning the error, so the next call (or rt_multi_destroy) starts from idle
// devices.  Errors here are ignored: the call is already failing.
int drain(rt_multi *m, int rc) {
  for (int g = 0; g < int(m->ctx.size()); g++)
    if (m->ctx[g]) {
      (void)hipSetDevice(m->dev(g));
      (void)hipStreamSynchronize(rtmi::ctx_stream(m->ctx[g]));
    }
  return rc;
}

struct KeepDevice {
  int prev = 0;
  KeepDevice() { (void)hipGetDevice(&prev); }
  ~KeepDevice() { (void)hipSetDevice(prev); }
};

// strips of nrows x W for the render that follows (reused when large enough)
int ensure_buffers(rt_multi *m, size_t strip_elems) {
  if (strip_elems > m->strip_cap) {
    for (int g = 0; g < m->G; g++) {
      (void)hipSetDevice(m->dev(g));
      if (m->strip[g]) (void)hipFree(m->strip[g]);
      m->strip[g] = nullptr;
      if (hipMalloc(&m->strip[g], strip_elems * sizeof(float)) != hipSuccess) {
        m->strip_cap = 0;
        return set_error(RT_ENOMEM, "strip allocation on GPU %d", g);
      }
    }
    m->strip_cap = strip_elems;
  }
  if (strip_elems * m->G > m->recv_cap) {
    (void)hipSetDevice(m->dev(0));
    if (m->recv) (void)hipFree(m->recv);
    m->recv = nullptr;
    if (hipMalloc(&m->recv, strip_elems * m->G * sizeof(float)) != hipSuccess) {
      m->recv_cap = 0;
      return set_error(RT_ENOMEM, "gather buffer on GPU 0");
    }
    m->recv_cap = strip_elems * m->G;
  }
  return RT_OK;
}

// RTMI_MULTI_MOCK_FAIL=g: the injected failure of logical device g (mock only)
int injected_failure(const rt_multi *m, int g, const char *what) {
  if (!m->mock) return RT_OK;
  const char *f = std::getenv("RTMI_MULTI_MOCK_FAIL");
  if (f && *f && std::atoi(f) == g) return set_error(RT_EHIP, "%s: injected failure on logical device %d (RTMI_MULTI_MOCK_FAIL)", what, g);
  return RT_OK;
}

// The mock's exchange step: each strip copied into device 0's receive buffer
// on device 0's stream, in rank order, after device 0 has waited for every
// strip (gather_unpermute_body) — what ncclGather does, with no communicator.
int mock_gather(rt_multi *m, size_t strip_elems, hipStream_t s0) {
  for (int g = 0; g < m->G; g++)
    if (hipMemcpyPeerAsync(m->recv + size_t(g) * strip_elems, m->dev(0), m->strip[g], m->dev(g),
                           strip_elems * sizeof(float), s0) != hipSuccess)
      return set_error(RT_EHIP, "mock gather copy of strip %d", g);
  return RT_OK;
}

// The single exchange step: every strip (already enqueued on its device's
// stream) to GPU 0, then rows un-permuted into the host image.
int gather_unpermute_body(rt_multi *m, int32_t W, int32_t H, int32_t nrows, float *sum) {
  const int G = m->G;
  const size_t strip_elems = size_t(nrows) * W * 3;
  std::vector<hipStream_t> streams(G);
  for (int g = 0; g < G; g++) streams[g] = rtmi::ctx_stream(m->ctx[g]);
  // device 0 starts the gather clock once every strip is rendered
  (void)hipSetDevice(m->dev(0));
  for (int g = 1; g < G; g++)
    if (hipStreamWaitEvent(streams[0], m->ev_end[g], 0) != hipSuccess) return set_error(RT_EHIP, "wait for GPU %d", g);
  if (hipEventRecord(m->gather_begin, streams[0]) != hipSuccess) return set_error(RT_EHIP, "gather event");
  if (m->mock) {
    if (int rc = mock_gather(m, strip_elems, streams[0])) return rc;
  } else {
    ncclResult_t r = ncclGroupStart();
    for (int g = 0; g < G && r == ncclSuccess; g++) {
      (void)hipSetDevice(g);
      r = ncclGather(m->strip[g], g == 0 ? m->recv : nullptr, strip_elems, ncclFloat, 0, m->comm[g], streams[g]);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) return set_error(RT_ERCCL, "ncclGather: %s", ncclGetErrorString(r));
  }
  (void)hipSetDevice(m->dev(0));
  if (hipEventRecord(m->gather_end, streams[0]) != hipSuccess) return set_error(RT_EHIP, "gather event");
  for (int g = 0; g < G; g++) {
    (void)hipSetDevice(m->dev(g));
    if (hipStreamSynchronize(streams[g]) != hipSuccess) return set_error(RT_EHIP, "sync GPU %d", g);
    if (m->mock) continue;
    ncclResult_t ae = ncclSuccess;
    ncclCommGetAsyncError(m->comm[g], &ae);
    if (ae != ncclSuccess) return set_error(RT_ERCCL, "RCCL async error on GPU %d: %s", g, ncclGetErrorString(ae));
  }
  m->strip_ms.assign(G, -1.0f);
  for (int g = 0; g < G; g++) {
    (void)hipSetDevice(m->dev(g));
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, m->ev_begin[g], m->ev_end[g]) == hipSuccess) m->strip_ms[g] = ms;
  }
  (void)hipSetDevice(m->dev(0));
  if (hipEventElapsedTime(&m->gather_ms, m->gather_begin, m->gather_end) != hipSuccess) m->gather_ms = -1.0f;
  m->host.resize(strip_elems * G);
  if (hipMemcpy(m->host.data(), m->recv, m->host.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(RT_EHIP, "gather buffer copy");
  return rt_unpermute_rows(m->host.data(), G, nrows, W, H, sum);
}
int gather_unpermute(rt_multi *m, int32_t W, int32_t H, int32_t nrows, float *sum) {
  const int rc = gather_unpermute_body(m, W, H, nrows, sum);
  return rc == RT_OK ? rc : drain(m, rc);
}
}  // namespace

RTMI_EXPORT int rt_multi_create(const rt_scene *scene, int32_t n_gpus, rt_multi **out) {
  if (!out) return set_error(RT_EINVAL, "rt_multi_create: null out");
  *out = nullptr;
  if (!scene || n_gpus < 0) return set_error(RT_EINVAL, "rt_multi_create: bad argument");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return set_error(RT_ENODEVICE, "no HIP device visible");
  const char *mk = std::getenv("RTMI_MULTI_MOCK");
  const bool mock = mk && *mk && *mk != '0';
  const int G = n_gpus == 0 ? count : n_gpus;
  if (G > count && !mock) return set_error(RT_ENODEVICE, "asked for %d GPUs, %d visible", G, count);
  KeepDevice keep;
  rt_multi *m = new rt_multi;
  m->G = G;
  m->visible = count;
  m->mock = mock;
  m->ctx.assign(G, nullptr);
  m->strip.assign(G, nullptr);
  m->ev_begin.assign(G, nullptr);
  m->ev_end.assign(G, nullptr);
  int rc = RT_OK;
  for (int g = 0; g < G && rc == RT_OK; g++) {
    if ((rc = rt_ctx_create(m->dev(g), &m->ctx[g])) || (rc = rt_ctx_set_scene(m->ctx[g], scene))) break;
    (void)hipSetDevice(m->dev(g));
    if (hipEventCreate(&m->ev_begin[g]) != hipSuccess || hipEventCreate(&m->ev_end[g]) != hipSuccess)
      rc = set_error(RT_EHIP, "events on GPU %d", g);
  }
  if (rc == RT_OK) {
    (void)hipSetDevice(m->dev(0));
    if (hipEventCreate(&m->gather_begin) != hipSuccess || hipEventCreate(&m->gather_end) != hipSuccess)
      rc = set_error(RT_EHIP, "gather events");
  }
  if (rc == RT_OK && !mock) {
    m->comm.assign(G, nullptr);
    std::vector<int> devs(G);
    for (int g = 0; g < G; g++) devs[g] = g;
    ncclResult_t r = ncclCommInitAll(m->comm.data(), G, devs.data());
    if (r != ncclSuccess) {
      m->comm.assign(G, nullptr);
      rc = set_error(RT_ERCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
  }
  if (rc != RT_OK) {
    destroy(m);
    return rc;
  }
  *out = m;
  return RT_OK;
}

RTMI_EXPORT int rt_multi_destroy(rt_multi *m) {
  KeepDevice keep;
  destroy(m);
  return RT_OK;
}

RTMI_EXPORT int rt_multi_device_count(rt_multi *m, int32_t *n) {
  if (!m || !n) return set_error(RT_EINVAL, "rt_multi_device_count: null");
  *n = m->G;
  return RT_OK;
}

RTMI_EXPORT int rt_multi_context(rt_multi *m, int32_t g, rt_ctx **ctx) {
  if (!m || !ctx || g < 0 || g >= m->G) return set_error(RT_EINVAL, "rt_multi_context: bad argument");
  *ctx = m->ctx[g];
  return RT_OK;
}

RTMI_EXPORT int rt_multi_render(rt_multi *m, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                                int32_t max_depth, uint64_t seed, float *sum) {
  if (!m || !cam || !sum || W < 2 || H < 2 || spp < 1) return set_error(RT_EINVAL, "rt_multi_render: bad argument");
  KeepDevice keep;
  const int G = m->G;
  const int32_t nrows = (H + G - 1) / G;
  int rc = ensure_buffers(m, size_t(nrows) * W * 3);
  // every strip enqueued on its own device's stream, then the gather
  for (int g = 0; g < G && rc == RT_OK; g++) {
    (void)hipSetDevice(m->dev(g));
    hipStream_t s = rtmi::ctx_stream(m->ctx[g]);
    if (hipEventRecord(m->ev_begin[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
    if (rc == RT_OK) rc = injected_failure(m, g, "rt_multi_render");
    if (rc == RT_OK) rc = rt_render_rows(m->ctx[g], cam, W, H, spp, max_depth, seed, g, G, nrows, m->strip[g], nullptr);
    (void)hipSetDevice(m->dev(g));
    if (rc == RT_OK && hipEventRecord(m->ev_end[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
  }
  if (rc != RT_OK) return drain(m, rc);  // earlier devices' strips may be in flight
  return gather_unpermute(m, W, H, nrows, sum);
}

RTMI_EXPORT int rt_multi_last_timing(rt_multi *m, float *strip_ms, float *gather_ms) {
  if (!m) return set_error(RT_EINVAL, "rt_multi_last_timing: null");
  if (m->strip_ms.size() != size_t(m->G)) return set_error(RT_EINVAL, "rt_multi_last_timing: no render yet");
  if (strip_ms) std::memcpy(strip_ms, m->strip_ms.data(), size_t(m->G) * sizeof(float));
  if (gather_ms) *gather_ms = m->gather_ms;
  return RT_OK;
}

RTMI_EXPORT int rt_multi_accum_reset(rt_multi *m, int32_t W, int32_t H) {
  if (!m || W < 2 || H < 2) return set_error(RT_EINVAL, "rt_multi_accum_reset: bad argument");
  KeepDevice keep;
  const int32_t nrows = (H + m->G - 1) / m->G;
  m->pass_W = 0;  // no valid accumulator set until every device has reset its own
  for (int g = 0; g < m->G; g++)
    if (int rc = rt_accum_reset(m->ctx[g], W, nrows)) return drain(m, rc);
  m->pass_W = W;
  m->pass_H = H;
  m->pass_nrows = nrows;
  return RT_OK;
}

RTMI_EXPORT int rt_multi_render_pass(rt_multi *m, const rt_camera *cam, int32_t s_begin, int32_t s_count,
                                     int32_t max_depth, uint64_t seed) {
  if (!m || !cam) return set_error(RT_EINVAL, "rt_multi_render_pass: bad argument");
  if (!m->pass_W) return set_error(RT_EINVAL, "rt_multi_render_pass: no accumulator (rt_multi_accum_reset)");
  KeepDevice keep;
  int rc = RT_OK;
  for (int g = 0; g < m->G && rc == RT_OK; g++) {
    (void)hipSetDevice(m->dev(g));
    hipStream_t s = rtmi::ctx_stream(m->ctx[g]);
    if (hipEventRecord(m->ev_begin[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
    if (rc == RT_OK) rc = injected_failure(m, g, "rt_multi_render_pass");
    if (rc == RT_OK)
      rc = rt_render_pass(m->ctx[g], cam, m->pass_W, m->pass_H, s_begin, s_count, max_depth, seed, g, m->G,
                          m->pass_nrows, nullptr);
    (void)hipSetDevice(m->dev(g));
    if (rc == RT_OK && hipEventRecord(m->ev_end[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
  }
  if (rc != RT_OK) {
    // devices 0..g-1 hold this pass's samples and the others do not: the
    // accumulators no longer cover one sample range, so resolving them would
    // return rows of different sample counts.  Invalid until the next reset.
    m->pass_W = 0;
    return drain(m, rc);
  }
  return RT_OK;
}

RTMI_EXPORT int rt_multi_accum_resolve(rt_multi *m, float *sum) {
  if (!m || !sum) return set_error(RT_EINVAL, "rt_multi_accum_resolve: bad argument");
  if (!m->pass_W) return set_error(RT_EINVAL, "rt_multi_accum_resolve: no accumulator (rt_multi_accum_reset)");
  KeepDevice keep;
  int rc = ensure_buffers(m, size_t(m->pass_nrows) * m->pass_W * 3);
  for (int g = 0; g < m->G && rc == RT_OK; g++) {
    (void)hipSetDevice(m->dev(g));
    hipStream_t s = rtmi::ctx_stream(m->ctx[g]);
    if (hipEventRecord(m->ev_begin[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
    if (rc == RT_OK) rc = injected_failure(m, g, "rt_multi_accum_resolve");
    if (rc == RT_OK) rc = rt_accum_resolve(m->ctx[g], m->strip[g], nullptr, nullptr);
    (void)hipSetDevice(m->dev(g));
    if (rc == RT_OK && hipEventRecord(m->ev_end[g], s) != hipSuccess) rc = set_error(RT_EHIP, "event on GPU %d", g);
  }
  if (rc != RT_OK) return drain(m, rc);
  return gather_unpermute(m, m->pass_W, m->pass_H, m->pass_nrows, sum);
}

RTMI_EXPORT int rt_render_multi(const rt_scene *scene, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                                int32_t max_depth, uint64_t seed, int32_t n_gpus, float *sum) {
  if (!scene || !cam || !sum || W < 2 || H < 2 || spp < 1 || n_gpus < 0)
    return set_error(RT_EINVAL, "rt_render_multi: bad argument");
  rt_multi *m = nullptr;
  int rc = rt_multi_create(scene, n_gpus, &m);
  if (rc == RT_OK) rc = rt_multi_render(m, cam, W, H, spp, max_depth, seed, sum);
  rt_multi_destroy(m);
  return rc;
}
