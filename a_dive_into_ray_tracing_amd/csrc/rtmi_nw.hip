// rtmi_nw.hip — gfx950 kernel and device C ABI of the Next-Week renderer
// (include/rtmi_nw.h).
//
// Same execution design as the RTIOW kernel (rtmi_device.hip render_kernel):
// one wavefront owns a work item = (8x8 pixel tile, range of samples); lanes
// pull (pixel, sample) jobs from a wave-local queue and regenerate paths as
// theirs terminate (__ballot + mbcnt compaction); colours are summed as int64
// fixed point in LDS, then one global atomic per pixel per item.  The
// reference (main.cu:125-145) instead gives each thread one pixel and loops
// all its samples, so a warp waits for its longest path at every sample.
// Per path segment: stackless BVH walk over the flattened objects (the
// reference walks a pointer tree of virtual hittables), deferred hit record
// of the winner, then texture lookup and scatter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>

#include "rtmi_internal.h"
#include "rtmi_nw_internal.h"
#include "rtmi_nw_path.h"

namespace rtmi {
namespace nw {

struct Args {
  Cam<float> cam;
  float time0, time1;
  int32_t W, H, spp, max_depth;
  uint64_t seed;
  int32_t row0, row_step, nrows_valid;
  int32_t tiles_x, tiles, chunk, nch, n_items;
};

constexpr int kWaves = 4;  // waves per block

__device__ __forceinline__ int64_t fixed(float c) { return int64_t(c * 4294967296.0f); }

template <bool CHUNKED>
__global__ __launch_bounds__(64 * kWaves) void render_kernel(View sc, Args a, unsigned long long *__restrict__ accum,
                                                             float *__restrict__ out,
                                                             unsigned long long *__restrict__ segments) {
  __shared__ unsigned long long acc[kWaves][3][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * kWaves + wave;
  if (item >= a.n_items) return;  // wave-uniform
  const int tile = item / a.nch;
  const int s0 = (item - tile * a.nch) * a.chunk;
  const int ns = min(a.chunk, a.spp - s0);
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int x0 = tx * 8, y0 = ty * 8;
  const int vw = min(8, a.W - x0), vh = min(8, a.nrows_valid - y0);
  const int nv = vw * vh;
  const int nq = nv * ns;

  acc[wave][0][lane] = 0;
  acc[wave][1][lane] = 0;
  acc[wave][2][lane] = 0;
  unsigned nseg = 0;

  V o, d, T;
  float time = 0.f;
  int px = 0, depth = 0;
  Xoro rng;
  // job q -> pixel q % nv, sample s0 + q / nv; camera ray main.cu:139-141
  auto start = [&](int q) {
    const int s = s0 + q / nv;
    px = q - (q / nv) * nv;
    const int ly = px / vw, lx = px - ly * vw;
    const int i = x0 + lx;
    const int j = a.row0 + (y0 + ly) * a.row_step;
    rng.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(s));
    float ju, jv;
    rng.pair(ju, jv);
    const float u = (float(i) + ju) / float(a.W);
    const float v = (float(j) + jv) / float(a.H);
    get_ray<true, float>(a.cam, u, v, rng, o, d);
    time = __builtin_fmaf(rng.uni(), a.time1 - a.time0, a.time0);  // camera.h:75-79
    T = mk(1.f, 1.f, 1.f);
    depth = 0;
  };

  bool active = lane < nq;
  if (active) start(lane);
  int next = 64;
  for (;;) {
    if (__ballot(active) == 0) break;
    bool done = false;
    V col = mk(0.f, 0.f, 0.f);
    if (active) {
      ++nseg;
      const uint64_t seg_key = sc.has_media ? rng.next() : 0ull;
      float t;
      int face;
      const int32_t k = hit_world_nw(sc, o, d, time, seg_key, t, face);
      if (k < 0) {  // background main.cu:92-99
        col = mk(T.x * sc.bg[0], T.y * sc.bg[1], T.z * sc.bg[2]);
        done = true;
      } else {
        const Obj ob = k < sc.nobj ? sc.obj[k] : sc.med[k - sc.nobj];
        const Rec rec = make_rec(sc, ob, o, d, time, t, face);
        const Mat m = sc.mat[rec.mat];
        V at, nd;
        if (m.kind == kDiffuseLight) {  // emitted, no scatter: main.cu:76-90
          col = mul3(T, tex_value(sc, m.tex, rec.u, rec.v, rec.p));
          done = true;
        } else if (!scatter_nw(sc, rec, d, rng, at, nd)) {
          done = true;  // absorbed: emitted() = 0
        } else {
          T = mul3(T, at);
          o = rec.p;
          d = nd;
          if (++depth >= a.max_depth) {  // main.cu:100: the background, unattenuated
            col = mk(sc.bg[0], sc.bg[1], sc.bg[2]);
            done = true;
          }
        }
      }
    }
    const unsigned long long m = __ballot(done);
    if (m) {
      if (done) {
        atomicAdd(&acc[wave][0][px], (unsigned long long)fixed(col.x));
        atomicAdd(&acc[wave][1][px], (unsigned long long)fixed(col.y));
        atomicAdd(&acc[wave][2][px], (unsigned long long)fixed(col.z));
        const int rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
        const int q = next + rank;
        if (q < nq) start(q);
        else active = false;
      }
      next += __popcll(m);
    }
  }
  // wave sum of segments (lanes' counts) -> one atomic
  unsigned long long ws = nseg;
  for (int off = 32; off > 0; off >>= 1) ws += __shfl_xor(ws, off);
  if (lane == 0) atomicAdd(segments, ws);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < nv) {
    const int ly = lane / vw, lx = lane - ly * vw;
    const size_t o3 = (size_t(y0 + ly) * size_t(a.W) + size_t(x0 + lx)) * 3;
    for (int c = 0; c < 3; ++c) {
      const unsigned long long v = acc[wave][c][lane];
      if constexpr (CHUNKED) atomicAdd(&accum[o3 + c], v);
      else out[o3 + c] = float((long long)v) * 0x1p-32f;
    }
  }
}

__global__ void finalize_kernel(const unsigned long long *__restrict__ acc, float *__restrict__ out, size_t n) {
  const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = float((long long)acc[i]) * 0x1p-32f;
}

}  // namespace nw
}  // namespace rtmi

// ===========================================================================
// host side
// ===========================================================================
using namespace rtmi;
using namespace rtmi::nw;

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return set_error(RT_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct rt_nw_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Obj *obj = nullptr;
  int32_t *obj_id = nullptr;
  Obj *med = nullptr;
  int32_t *med_id = nullptr;
  int32_t nmed = 0;
  Inst *inst = nullptr;
  Mat *mat = nullptr;
  Tex *tex = nullptr;
  float4 *pvec = nullptr;
  int32_t *pperm = nullptr;
  uint8_t *img = nullptr;
  Image *imgd = nullptr;
  Node *nodes = nullptr;
  int32_t nobj = 0, nnodes = 0, ninst = 0, nmat = 0, ntex = 0;
  float bg[3] = {0.f, 0.f, 0.f};
  int32_t has_media = 0;
  unsigned long long *accum = nullptr;
  size_t accum_cap = 0;
  float *scratch = nullptr;
  size_t scratch_cap = 0;
  unsigned long long *segments = nullptr;
};

namespace {

struct Guard {
  int prev = -1;
  explicit Guard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~Guard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class T> int alloc_copy(T **p, const T *src, size_t count) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  const size_t n = count ? count : 1;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), n * sizeof(T));
  if (e != hipSuccess) return set_error(RT_ENOMEM, "hipMalloc(%zu B): %s", n * sizeof(T), hipGetErrorString(e));
  if (count && src) {
    e = hipMemcpy(*p, src, count * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) return set_error(RT_EHIP, "hipMemcpy: %s", hipGetErrorString(e));
  }
  return RT_OK;
}

Cam<float> camf(const rt_camera &c) {
  auto v = [](const double *p) { return mk(float(p[0]), float(p[1]), float(p[2])); };
  return Cam<float>{v(c.origin), v(c.lower_left_corner), v(c.horizontal), v(c.vertical), v(c.u), v(c.v),
                    float(c.lens_radius)};
}

View view_of(const rt_nw_ctx *c) {
  View v;
  v.obj = c->obj;
  v.obj_id = c->obj_id;
  v.med = c->med;
  v.med_id = c->med_id;
  v.nobj = c->nobj;
  v.nmed = c->nmed;
  v.inst = c->inst;
  v.mat = c->mat;
  v.tex = c->tex;
  v.perlin_vec = c->pvec;
  v.perlin_perm = c->pperm;
  v.image_px = c->img;
  v.image = c->imgd;
  v.nodes = c->nodes;
  v.nnodes = c->nnodes;
  for (int i = 0; i < 3; ++i) v.bg[i] = c->bg[i];
  v.has_media = c->has_media;
  return v;
}

}  // namespace

RTMI_EXPORT int rt_nw_ctx_create(int32_t device, rt_nw_ctx **out) {
  if (!out) return set_error(RT_EINVAL, "null out");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return set_error(RT_ENODEVICE, "no HIP device visible");
  if (device < 0 || device >= count) return set_error(RT_ENODEVICE, "device %d out of range [0,%d)", device, count);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(RT_ENODEVICE, "device %d is %s; librtmi is built for gfx950 only", device, prop.gcnArchName);
  Guard g(device);
  auto ctx = std::make_unique<rt_nw_ctx>();
  ctx->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  if (int rc = alloc_copy<unsigned long long>(&ctx->segments, nullptr, 1)) return rc;
  HIP_TRY(hipMemset(ctx->segments, 0, sizeof(unsigned long long)));
  *out = ctx.release();
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_destroy(rt_nw_ctx *ctx) {
  if (!ctx) return RT_OK;
  Guard g(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (void *p : {(void *)ctx->obj, (void *)ctx->obj_id, (void *)ctx->med, (void *)ctx->med_id, (void *)ctx->inst, (void *)ctx->mat, (void *)ctx->tex,
                  (void *)ctx->pvec, (void *)ctx->pperm, (void *)ctx->img, (void *)ctx->imgd, (void *)ctx->nodes,
                  (void *)ctx->accum, (void *)ctx->scratch, (void *)ctx->segments})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_set_scene(rt_nw_ctx *ctx, rt_nw_scene *s) {
  if (!ctx || !s) return set_error(RT_EINVAL, "rt_nw_ctx_set_scene: null");
  DeviceScene ds;
  if (int rc = build_device_scene(s, ds)) return rc;
  // every index the kernel follows is checked here, once
  const int32_t nt = int32_t(ds.tex.size()), nm = int32_t(ds.mat.size()), ni = int32_t(ds.inst.size());
  const int32_t np = int32_t(ds.perlin_perm.size() / (3 * kPerlinN)), nim = int32_t(ds.image.size());
  for (const Obj &o : ds.obj)
    if (o.mat < 0 || o.mat >= nm || o.inst >= ni || o.kind < kSphere || o.kind > kBox || o.aux < 0 ||
        o.aux > int32_t(ds.med.size()))
      return set_error(RT_EINVAL, "rt_nw: object with bad material/instance/kind");
  for (const Obj &o : ds.med) {
    const int bk = o.aux & 255, ns = o.aux >> 8;
    if (o.mat < 0 || o.mat >= nm || o.inst >= ni || o.kind != kMedium || (bk != kSphere && bk != kMovingSphere && bk != kBox) ||
        ns < 1 || ns > 8)
      return set_error(RT_EINVAL, "rt_nw: bad medium record");
  }
  for (const Mat &m : ds.mat)
    if (m.kind != kDielectric && (m.tex < 0 || m.tex >= nt)) return set_error(RT_EINVAL, "rt_nw: material with bad texture");
  for (const Tex &t : ds.tex) {
    if (t.kind == kChecker && (t.a < 0 || t.a >= nt || t.b < 0 || t.b >= nt)) return set_error(RT_EINVAL, "rt_nw: bad checker");
    if (t.kind == kNoise && (t.a < 0 || t.a >= np)) return set_error(RT_EINVAL, "rt_nw: bad perlin index");
    if (t.kind == kImage && (t.a < 0 || t.a >= nim)) return set_error(RT_EINVAL, "rt_nw: bad image index");
  }
  std::vector<float4> pv(ds.perlin_vec.size() / 4);
  std::memcpy(pv.data(), ds.perlin_vec.data(), pv.size() * sizeof(float4));
  Guard g(ctx->device);
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  int rc;
  if ((rc = alloc_copy(&ctx->obj, ds.obj.data(), ds.obj.size())) ||
      (rc = alloc_copy(&ctx->med, ds.med.data(), ds.med.size())) ||
      (rc = alloc_copy(&ctx->med_id, ds.med_id.data(), ds.med_id.size())) ||
      (rc = alloc_copy(&ctx->obj_id, ds.obj_id.data(), ds.obj_id.size())) ||
      (rc = alloc_copy(&ctx->inst, ds.inst.data(), ds.inst.size())) ||
      (rc = alloc_copy(&ctx->mat, ds.mat.data(), ds.mat.size())) ||
      (rc = alloc_copy(&ctx->tex, ds.tex.data(), ds.tex.size())) || (rc = alloc_copy(&ctx->pvec, pv.data(), pv.size())) ||
      (rc = alloc_copy(&ctx->pperm, ds.perlin_perm.data(), ds.perlin_perm.size())) ||
      (rc = alloc_copy(&ctx->img, ds.image_px.data(), ds.image_px.size())) ||
      (rc = alloc_copy(&ctx->imgd, ds.image.data(), ds.image.size())) ||
      (rc = alloc_copy(&ctx->nodes, ds.nodes.data(), ds.nodes.size())))
    return rc;
  ctx->nobj = int32_t(ds.obj.size());
  ctx->nmed = int32_t(ds.med.size());
  ctx->nnodes = int32_t(ds.nodes.size());
  ctx->ninst = ni;
  ctx->nmat = nm;
  ctx->ntex = nt;
  for (int c = 0; c < 3; ++c) ctx->bg[c] = ds.background[c];
  ctx->has_media = ds.has_media ? 1 : 0;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_info(rt_nw_ctx *ctx, int32_t *n_prims, int32_t *n_nodes) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (n_prims) *n_prims = ctx->nobj + ctx->nmed;
  if (n_nodes) *n_nodes = ctx->nnodes;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_render_rows(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t spp,
                                  int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows,
                                  float *dev_strip, void *stream) {
  if (!ctx || !cam || !dev_strip) return set_error(RT_EINVAL, "rt_nw_render_rows: null argument");
  if (ctx->nobj + ctx->nmed <= 0) return set_error(RT_EINVAL, "no scene uploaded (rt_nw_ctx_set_scene)");
  if (W < 1 || H < 1 || spp < 1 || spp >= (1 << 24) || max_depth < 1 || int64_t(W) * H >= (int64_t(1) << 40))
    return set_error(RT_EINVAL, "rt_nw_render_rows: bad size (W, H, spp >= 1, spp < 2^24, max_depth >= 1)");
  if (nrows < 1 || row_step < 1 || row0 < 0 || row0 >= H) return set_error(RT_EINVAL, "rt_nw_render_rows: bad row set");
  if (!(cam->time0 >= 0.0 && cam->time1 <= 1.0 && cam->time0 <= cam->time1))
    return set_error(RT_EINVAL, "rt_nw_render_rows: shutter must lie in [0, 1]");
  const int32_t valid = std::min<int64_t>(nrows, (int64_t(H) - 1 - row0) / row_step + 1);
  Guard g(ctx->device);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  Args a;
  a.cam = camf(cam->cam);
  a.time0 = float(cam->time0);
  a.time1 = float(cam->time1);
  a.W = W;
  a.H = H;
  a.spp = spp;
  a.max_depth = max_depth;
  a.seed = seed;
  a.row0 = row0;
  a.row_step = row_step;
  a.nrows_valid = valid;
  a.tiles_x = (W + 7) / 8;
  a.tiles = a.tiles_x * ((valid + 7) / 8);
  a.chunk = std::min(spp, 32);
  a.nch = (spp + a.chunk - 1) / a.chunk;
  if (int64_t(a.tiles) * a.nch >= (int64_t(1) << 31) - kWaves) return set_error(RT_EINVAL, "render too large");
  a.n_items = a.tiles * a.nch;
  if (valid < nrows)  // rows past H: zero
    HIP_TRY(hipMemsetAsync(dev_strip + size_t(valid) * W * 3, 0, size_t(nrows - valid) * W * 3 * sizeof(float), st));
  HIP_TRY(hipMemsetAsync(ctx->segments, 0, sizeof(unsigned long long), st));
  const unsigned blocks = unsigned((a.n_items + kWaves - 1) / kWaves);
  const View v = view_of(ctx);
  if (a.nch > 1) {
    const size_t nv = size_t(valid) * W * 3;
    if (nv > ctx->accum_cap) {
      HIP_TRY(hipStreamSynchronize(st));
      if (int rc = alloc_copy<unsigned long long>(&ctx->accum, nullptr, nv)) return rc;
      ctx->accum_cap = nv;
    }
    HIP_TRY(hipMemsetAsync(ctx->accum, 0, nv * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(render_kernel<true>, dim3(blocks), dim3(64 * kWaves), 0, st, v, a, ctx->accum, dev_strip,
                       ctx->segments);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(finalize_kernel, dim3(unsigned((nv + 255) / 256)), dim3(256), 0, st, ctx->accum, dev_strip, nv);
  } else {
    hipLaunchKernelGGL(render_kernel<false>, dim3(blocks), dim3(64 * kWaves), 0, st, v, a, ctx->accum, dev_strip,
                       ctx->segments);
  }
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

RTMI_EXPORT int rt_nw_render(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t spp,
                             int32_t max_depth, uint64_t seed, float *sum) {
  if (!ctx || !sum) return set_error(RT_EINVAL, "rt_nw_render: null argument");
  if (W < 1 || H < 1 || int64_t(W) * H >= (int64_t(1) << 40)) return set_error(RT_EINVAL, "rt_nw_render: bad size");
  Guard g(ctx->device);
  const size_t n = size_t(W) * size_t(H) * 3;
  if (n > ctx->scratch_cap) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (int rc = alloc_copy<float>(&ctx->scratch, nullptr, n)) return rc;
    ctx->scratch_cap = n;
  }
  if (int rc = rt_nw_render_rows(ctx, cam, W, H, spp, max_depth, seed, 0, 1, H, ctx->scratch, ctx->stream)) return rc;
  HIP_TRY(hipMemcpyAsync(sum, ctx->scratch, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_last_segments(rt_nw_ctx *ctx, uint64_t *segments) {
  if (!ctx || !segments) return set_error(RT_EINVAL, "null");
  Guard g(ctx->device);
  unsigned long long v = 0;
  HIP_TRY(hipDeviceSynchronize());  // the render may have run on a caller's stream
  HIP_TRY(hipMemcpy(&v, ctx->segments, sizeof v, hipMemcpyDeviceToHost));
  *segments = v;
  return RT_OK;
}
