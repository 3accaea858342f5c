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
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <type_traits>

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

// Two kernel shapes, the same per-path arithmetic (bit-identical images):
//  * persistent (default when the scene fits in LDS): one 16-wave block per
//    CU stages the BVH nodes — and the objects, when they fit too — into LDS
//    once for the whole launch; its waves pull work items from a global
//    counter, so no wave waits for a slow item of another;
//  * grid: one wave per work item in 4-wave blocks, nodes in LDS when they
//    fit the per-block budget (several blocks per CU), else in global memory.
// Measured (profiles/r01/nw): 4-wave grid blocks beat 8-wave ones (a block's
// LDS stays allocated until its slowest item ends), LDS nodes +23% and LDS
// objects +13% on the motion-blur scene.
#ifndef RTMI_NW_WAVES
#define RTMI_NW_WAVES 4
#endif
#ifndef RTMI_NW_LDS_KB
#define RTMI_NW_LDS_KB 34
#endif
#ifndef RTMI_NW_PERSIST
#define RTMI_NW_PERSIST 1
#endif
#ifndef RTMI_NW_LDS_OBJS
#define RTMI_NW_LDS_OBJS 1
#endif
constexpr int kWaves = RTMI_NW_WAVES;                         // grid kernel: waves per block
constexpr size_t kLdsBudget = size_t(RTMI_NW_LDS_KB) * 1024;  // grid kernel: staged bytes per block
constexpr int kPWaves = 16;                                   // persistent kernel: waves per block (one per CU)
// spheres-only instantiation of the persistent kernel: waves per block and
// the minimum waves per SIMD it is compiled for (VGPR budget 512 / per_eu).
// Motion-blur scene 1200x800x500 (profiles/r02/ab_nw_spheres_only/): general
// kernel 100.6 ms; spheres-only at 89 VGPRs (4 waves per SIMD) 79.2;
// 8-wave blocks at 6 per SIMD (80 VGPRs, 7 spilled) 63.8; 16- or 8-wave
// blocks at 8 per SIMD (64 VGPRs, spills) 60.4-60.5
#ifndef RTMI_NW_SIMPLE_WAVES
#define RTMI_NW_SIMPLE_WAVES 16
#endif
#ifndef RTMI_NW_SIMPLE_PER_EU
#define RTMI_NW_SIMPLE_PER_EU 8
#endif
template <bool S> constexpr int persist_waves() { return S ? RTMI_NW_SIMPLE_WAVES : kPWaves; }
// minimum waves per SIMD of the general persistent kernel's BVH
// instantiations: 8 (64 VGPRs, spills) lets two 16-wave blocks share a CU
// when the staged bytes allow it.  Final scene at 1024 spp
// (profiles/r02/ab_nw_occupancy/): nodes + objects in LDS, one block per CU
// (100 VGPRs) 1 062 ms; objects in global memory, one block 1 185; objects
// in global memory, two blocks at 64 VGPRs 1 009-1 013.
#ifndef RTMI_NW_PERSIST_PER_EU
#define RTMI_NW_PERSIST_PER_EU 8
#endif
// Dynamic LDS budgets of the persistent kernel, derived from its static LDS
// (the waves' accumulators and the camera, rounded up to the allocation
// granule): staged bytes (nodes, and objects when they fit) that leave room
// for two blocks per CU, and for one (160 KB LDS per CU).  The launch path
// also checks the kernel's actual static size (hipFuncGetAttributes), so a
// new __shared__ variable cannot silently push a block past the CU.
constexpr size_t kCuLds = 160 * 1024;
constexpr size_t kPStaticLds = (sizeof(unsigned long long) * 3 * 64 * kPWaves + 23 * sizeof(float) + 255) / 256 * 256;
constexpr size_t kPTwoBlockBudget = kCuLds / 2 - kPStaticLds;
constexpr size_t kPLdsBudget = kCuLds - kPStaticLds;

// RTMI_NW_PHASES builds (analysis only): wave-level cycles (s_memtime) of a
// work item's loop passes: [0] closest hit, [1] hit record + texture +
// scatter, [2] accumulation + regeneration, [3] whole item; read with
// rt_nw_debug_phases.
#ifndef RTMI_NW_PHASES
#define RTMI_NW_PHASES 0
#endif
#if RTMI_NW_PHASES
__device__ unsigned long long g_nw_phase[4];
#endif
#if RTMI_STATS
// RTMI_STATS build: executed work of the launches since the last
// rt_nw_debug_counters call — FLOP, node visits, object tests, cell steps
__device__ unsigned long long g_nw_stats[4];
#endif

// NaN -> 0, clamped to [0, 64]: as rtmi_device.hip to_fixed (and the oracle)
__device__ __forceinline__ int64_t fixed(float c) {
  const float g = c == c ? __builtin_amdgcn_fmed3f(c, 0.0f, 64.0f) : 0.0f;  // branch-free guard
  const uint32_t hi = uint32_t(g);
  const uint32_t lo = uint32_t((g - float(hi)) * 4294967296.0f);
  return int64_t((uint64_t(hi) << 32) | lo);
}

// The camera, shutter and image size in LDS (23 floats), read at each
// regeneration: the kernel's scalar registers otherwise overflow and the
// compiler parks them in VGPR lanes (v_readlane at every regeneration), as in
// the RTIOW kernel.  Staged before stage_scene's barrier.
__device__ __forceinline__ void stage_camera(float *cl, const Args &a) {
  const unsigned t = threadIdx.x;
  if (t < 23) {
    float v;
    switch (t / 3) {
      case 0: v = (&a.cam.origin.x)[t % 3]; break;
      case 1: v = (&a.cam.llc.x)[t % 3]; break;
      case 2: v = (&a.cam.hor.x)[t % 3]; break;
      case 3: v = (&a.cam.ver.x)[t % 3]; break;
      case 4: v = (&a.cam.u.x)[t % 3]; break;
      case 5: v = (&a.cam.v.x)[t % 3]; break;
      default:
        v = t == 18 ? a.cam.lens : t == 19 ? a.time0 : t == 20 ? a.time1 - a.time0 : t == 21 ? float(a.W) : float(a.H);
        break;
    }
    cl[t] = v;
  }
}

template <bool LDS_NODES, bool LDS_OBJS, bool GRID>
__device__ __forceinline__ void stage_scene(const View &sc) {
  if constexpr (GRID) {  // objects, insertion indices, cell starts, refs, brute-force list (nw_grid_lds_bytes)
    const float4 *src = reinterpret_cast<const float4 *>(sc.obj);
    for (int i = threadIdx.x; i < 3 * sc.nobj; i += blockDim.x) nw_nodes_lds[i] = src[i];
    int32_t *ids = reinterpret_cast<int32_t *>(nw_nodes_lds + 3 * sc.nobj);
    for (int i = threadIdx.x; i < sc.nobj; i += blockDim.x) ids[i] = sc.obj_id[i];
    uint16_t *u = reinterpret_cast<uint16_t *>(ids + sc.nobj);
    const int nstart = sc.grid.ncells + 1;
    for (int i = threadIdx.x; i < nstart; i += blockDim.x) u[i] = sc.grid.cell_start[i];
    for (int i = threadIdx.x; i < sc.grid.nrefs; i += blockDim.x) u[nstart + i] = sc.grid.refs[i];
    int32_t *big = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(u) + ((size_t(nstart) + sc.grid.nrefs) * 2 + 3) / 4 * 4);
    for (int i = threadIdx.x; i < sc.nbig; i += blockDim.x) big[i] = sc.gbig[i];
    __syncthreads();
  } else if constexpr (LDS_NODES) {  // BVH nodes (lo[], hi[]), then objects and their insertion indices
    for (int i = threadIdx.x; i < sc.nnodes; i += blockDim.x) {
      nw_nodes_lds[i] = sc.nlo[i];
      nw_nodes_lds[sc.nnodes + i] = sc.nhi[i];
    }
    if constexpr (LDS_OBJS) {
      const float4 *src = reinterpret_cast<const float4 *>(sc.obj);
      float4 *dst = nw_nodes_lds + 2 * sc.nnodes;
      for (int i = threadIdx.x; i < 3 * sc.nobj; i += blockDim.x) dst[i] = src[i];
      int32_t *ids = reinterpret_cast<int32_t *>(dst + 3 * sc.nobj);
      for (int i = threadIdx.x; i < sc.nobj; i += blockDim.x) ids[i] = sc.obj_id[i];
    }
    __syncthreads();
  }
}

// One work item = (8x8 tile, <= chunk samples) on one wave: lanes pull
// (pixel, sample) jobs from the item's queue and regenerate paths as theirs
// end; sums in the wave's LDS accumulator, then one global add per pixel.
template <bool CHUNKED, bool LDS_NODES, bool LDS_OBJS, bool GRID, bool S = false>
__device__ __forceinline__ void run_item(const View &sc, const Args &a, int item, int lane,
                                         unsigned long long (&acc)[3][64], unsigned long long *__restrict__ accum,
                                         float *__restrict__ out, unsigned &nseg, const float *cl) {
  const int tile = item / a.nch;
  const int s0 = (item - tile * a.nch) * a.chunk;
  const int ns = min(a.chunk, a.spp - s0);
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int x0 = tx * 8, y0 = ty * 8;
  const int vw = min(8, a.W - x0), vh = min(8, a.nrows_valid - y0);
  const int nv = vw * vh;
  const int nq = nv * ns;

  acc[0][lane] = 0;
  acc[1][lane] = 0;
  acc[2][lane] = 0;

  V o, d, T;
  float time = 0.f;
  // the path's pixel in the tile (bits 24..29) and its depth (bits 0..23;
  // max_depth < 2^24 is checked on the host) in one register
  int pxd = 0;
  Xoro rng;
  // job q -> pixel q % nv, sample s0 + q / nv; camera ray main.cu:139-141.
  // Grid kernels: q / d = umulhi(2q, ceil(2^31 / d)), exact for d <= 64,
  // q < 2^25 (the RTIOW kernel's job decode, tests/test_kernel_arith.py;
  // chunk <= 65535 keeps q < 2^22) — a multiply instead of the 32-bit division
  // expansion (motion blur 59.5 -> 58.1 ms); the BVH kernel keeps the division
  // (its two multipliers cost more registers than they save: final scene
  // 283.6 -> 286.2 ms at 256 spp, profiles/r03/ab_nw_jobdiv.txt)
  constexpr bool kMulDiv = GRID;
  const uint32_t m_nv = 0x7FFFFFFFu / uint32_t(max(nv, 1)) + 1u, m_vw = 0x7FFFFFFFu / uint32_t(vw) + 1u;
  auto start = [&](int q) {
    const int qs = kMulDiv ? int(__umulhi(uint32_t(q) << 1, m_nv)) : q / nv;
    const int s = s0 + qs;
    const int px = q - qs * nv;
    const int ly = kMulDiv ? int(__umulhi(uint32_t(px) << 1, m_vw)) : px / vw, lx = px - ly * vw;
    const int i = x0 + lx;
    const int j = a.row0 + (y0 + ly) * a.row_step;
    rng.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(s));
    float ju, jv;
    rng.pair(ju, jv);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // read here, not hoisted out of the loop
    const float u = (float(i) + ju) / cl[21];
    const float v = (float(j) + jv) / cl[22];
    Cam<float> cm;
    cm.origin = mk(cl[0], cl[1], cl[2]);
    cm.llc = mk(cl[3], cl[4], cl[5]);
    cm.hor = mk(cl[6], cl[7], cl[8]);
    cm.ver = mk(cl[9], cl[10], cl[11]);
    cm.u = mk(cl[12], cl[13], cl[14]);
    cm.v = mk(cl[15], cl[16], cl[17]);
    cm.lens = cl[18];
    get_ray<true, float>(cm, u, v, rng, o, d);
    time = __builtin_fmaf(rng.uni(), cl[20], cl[19]);  // camera.h:75-79
    T = mk(1.f, 1.f, 1.f);
    pxd = px << 24;
  };

#if RTMI_NW_PHASES
  unsigned long long ph[4] = {0, 0, 0, 0}, pa = 0, pb = 0;
  const unsigned long long p_start = __builtin_amdgcn_s_memtime();
#endif
  NwCount cnt{0, 0, 0, 0};
  bool active = lane < nq;
  if (active) start(lane);
  int next = 64;
  for (;;) {
    const unsigned long long live = __ballot(active);
    if (live == 0) break;
    nseg = unsigned(__builtin_amdgcn_readfirstlane(int(nseg + unsigned(__popcll(live)))));
    bool done = false;
    V col = mk(0.f, 0.f, 0.f);
#if RTMI_NW_PHASES
    pa = __builtin_amdgcn_s_memtime();
#endif
    if (active) {
      const uint64_t seg_key = !S && sc.has_media ? rng.next() : 0ull;
      float t;
      int face;
      const int32_t k = GRID ? hit_world_nw_grid<S>(sc, o, d, time, seg_key, t, face, &cnt)
                             : hit_world_nw<LDS_NODES, LDS_OBJS>(sc, o, d, time, seg_key, t, face, &cnt);
#if RTMI_NW_PHASES
      pb = __builtin_amdgcn_s_memtime();
#endif
      if (k < 0) {  // background main.cu:92-99
        col = mk(T.x * sc.bg[0], T.y * sc.bg[1], T.z * sc.bg[2]);
        done = true;
      } else {
        const Rec rec = S || k < sc.nobj ? make_rec<S>(sc, sc.obj[k], o, d, time, t, face)
                                         : make_rec_medium(sc, sc.med[k - sc.nobj], o, d, time);
        const Mat m = sc.mat[rec.mat];
        V at, nd;
        if (m.kind == kDiffuseLight) {  // emitted, no scatter: main.cu:76-90
          col = mul3(T, tex_value<S>(sc, m.tex, rec.u, rec.v, rec.p));
          done = true;
        } else if (!scatter_nw<S>(sc, rec, d, rng, at, nd)) {
          done = true;  // absorbed: emitted() = 0
        } else {
          T = mul3(T, at);
          o = rec.p;
          d = nd;
          if ((++pxd & 0xFFFFFF) >= a.max_depth) {  // main.cu:100: the background, unattenuated
            col = mk(sc.bg[0], sc.bg[1], sc.bg[2]);
            done = true;
          }
        }
      }
    }
#if RTMI_NW_PHASES
    const unsigned long long pc = __builtin_amdgcn_s_memtime();
    pb = __shfl(pb, __builtin_ctzll(__ballot(active)));  // (set by the lanes that ran the hit)
    ph[0] += pb - pa;
    ph[1] += pc - pb;
#endif
    const unsigned long long m = __ballot(done);
    if (m) {
      if (done) {
        const int px = pxd >> 24;
        atomicAdd(&acc[0][px], (unsigned long long)fixed(col.x));
        atomicAdd(&acc[1][px], (unsigned long long)fixed(col.y));
        atomicAdd(&acc[2][px], (unsigned long long)fixed(col.z));
        const int rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
        const int q = next + rank;
        if (q < nq) start(q);
        else active = false;
      }
      next = __builtin_amdgcn_readfirstlane(next + int(__popcll(m)));
    }
#if RTMI_NW_PHASES
    ph[2] += __builtin_amdgcn_s_memtime() - pc;
#endif
  }
#if RTMI_NW_PHASES
  ph[3] = __builtin_amdgcn_s_memtime() - p_start;
  if (lane == __builtin_ctzll(__ballot(1)))
    for (int q = 0; q < 4; ++q) atomicAdd(&g_nw_phase[q], ph[q]);
#endif
#if RTMI_STATS
  atomicAdd(&g_nw_stats[0], cnt.flop);
  atomicAdd(&g_nw_stats[1], (unsigned long long)cnt.nodes);
  atomicAdd(&g_nw_stats[2], (unsigned long long)cnt.objects);
  atomicAdd(&g_nw_stats[3], (unsigned long long)cnt.cells);
#else
  (void)cnt;
#endif
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < nv) {
    const int ly = lane / vw, lx = lane - ly * vw;
    const size_t o3 = (size_t(y0 + ly) * size_t(a.W) + size_t(x0 + lx)) * 3;
    for (int c = 0; c < 3; ++c) {
      const unsigned long long v = acc[c][lane];
      if constexpr (CHUNKED) atomicAdd(&accum[o3 + c], v);
      else out[o3 + c] = float((long long)v) * 0x1p-32f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void add_segments(unsigned nseg, int lane, unsigned long long *segments) {
  if (lane == 0) atomicAdd(segments, (unsigned long long)nseg);  // the wave's world.hit calls (wave-uniform)
}

template <bool CHUNKED, bool LDS_NODES, bool LDS_OBJS, bool GRID>
__global__ __launch_bounds__(64 * kWaves) void render_kernel(View sc, Args a, unsigned long long *__restrict__ accum,
                                                             float *__restrict__ out,
                                                             unsigned long long *__restrict__ segments) {
  __shared__ unsigned long long acc[kWaves][3][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * kWaves + wave;
  __shared__ float cam_lds[23];
  stage_camera(cam_lds, a);
  if constexpr (!LDS_NODES && !GRID) __syncthreads();  // (stage_scene's barrier covers the others)
  stage_scene<LDS_NODES, LDS_OBJS, GRID>(sc);  // block barrier inside: before any wave leaves
  if (item >= a.n_items) return;         // wave-uniform
  unsigned nseg = 0;
  run_item<CHUNKED, LDS_NODES, LDS_OBJS, GRID>(sc, a, item, lane, acc[wave], accum, out, nseg, cam_lds);
  add_segments(nseg, lane, segments);
}

#ifndef RTMI_NW_PERSIST_GRID_PER_EU
#define RTMI_NW_PERSIST_GRID_PER_EU 1
#endif
template <bool CHUNKED, bool LDS_OBJS, bool GRID, bool S = false>
__global__ __launch_bounds__(64 * persist_waves<S>(), S ? RTMI_NW_SIMPLE_PER_EU : (GRID ? RTMI_NW_PERSIST_GRID_PER_EU : RTMI_NW_PERSIST_PER_EU)) void render_persistent(View sc, Args a,
                                                                  unsigned long long *__restrict__ accum,
                                                                  float *__restrict__ out,
                                                                  unsigned long long *__restrict__ segments,
                                                                  unsigned *__restrict__ counter) {
  __shared__ unsigned long long acc[persist_waves<S>()][3][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ float cam_lds[23];
  stage_camera(cam_lds, a);
  stage_scene<true, LDS_OBJS, GRID>(sc);  // (its barrier covers the camera)
  unsigned nseg = 0;
  for (;;) {  // every wave leaves when the counter passes n_items
    unsigned it = 0;
    if (lane == 0) it = atomicAdd(counter, 1u);
    it = __builtin_amdgcn_readfirstlane(__shfl(it, 0));
    if (int(it) >= a.n_items) break;
    run_item<CHUNKED, true, LDS_OBJS, GRID, S>(sc, a, int(it), lane, acc[wave], accum, out, nseg, cam_lds);
  }
  add_segments(nseg, lane, segments);
}

// Debug (parity investigations): the segments of ONE camera sample (pixel
// i, j, sample s): per segment o.xyz, d.xyz, t, winner insertion index (as
// float bits) — the oracle's or_nw_trace records the same.
__global__ void trace_kernel(View sc, Args a, int i, int j, int s, float *rec, int cap, int *n_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Xoro rng;
  rng.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(s));
  float ju, jv;
  rng.pair(ju, jv);
  V o, d;
  get_ray<true, float>(a.cam, (float(i) + ju) / float(a.W), (float(j) + jv) / float(a.H), rng, o, d);
  const float time = __builtin_fmaf(rng.uni(), a.time1 - a.time0, a.time0);
  int n = 0;
  // the walk's work counters (written only by the RTMI_STATS build, which
  // would otherwise dereference a null counter pointer here)
  NwCount tcnt{0, 0, 0, 0};
  for (int depth = 0; depth < a.max_depth && n < cap; ++depth) {
    const uint64_t seg_key = sc.has_media ? rng.next() : 0ull;
    float t;
    int face;
    const int32_t k = hit_world_nw<false, false>(sc, o, d, time, seg_key, t, face, &tcnt);
    float *r = rec + 12 * n++;
    r[0] = o.x; r[1] = o.y; r[2] = o.z; r[3] = d.x; r[4] = d.y; r[5] = d.z; r[6] = t;
    r[7] = __int_as_float(k < 0 ? -1 : k < sc.nobj ? sc.obj_id[k] : sc.med_id[k - sc.nobj]);
    r[8] = r[9] = r[10] = 0.f;
    r[11] = __int_as_float(face);
    if (k < 0) break;
    const Rec rc = k < sc.nobj ? make_rec(sc, sc.obj[k], o, d, time, t, face) : make_rec_medium(sc, sc.med[k - sc.nobj], o, d, time);
    r[8] = rc.n.x; r[9] = rc.n.y; r[10] = rc.n.z;
    const Mat m = sc.mat[rc.mat];
    V at, nd;
    if (m.kind == kDiffuseLight || !scatter_nw(sc, rc, d, rng, at, nd)) break;
    o = rc.p;
    d = nd;
  }
  *n_out = n;
}

__global__ void finalize_kernel(const unsigned long long *__restrict__ acc, float *__restrict__ out, size_t n) {
  const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = float((long long)acc[i]) * 0x1p-32f;
}

// Closest hit of n given rays through the walk the renders use (validation:
// rt_nw_debug_hits): the uniform grid staged in LDS as the grid kernels stage
// it (GRID), or the BVH from global memory.  rays: {o.xyz, d.xyz, time, -} per
// ray; keys: the segments' medium keys (null: 0).
template <bool GRID>
__global__ __launch_bounds__(256) void debug_hits_kernel(View sc, const float *__restrict__ rays,
                                                         const unsigned long long *__restrict__ keys, int32_t n,
                                                         int32_t *__restrict__ out_id, float *__restrict__ out_t,
                                                         int32_t *__restrict__ out_face) {
  stage_scene<false, false, GRID>(sc);  // (GRID: ends with the block barrier, before any thread leaves)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float *r = rays + 8 * size_t(i);
  const V o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
  NwCount cnt{0, 0, 0, 0};
  float t;
  int face;
  const int32_t k = GRID ? hit_world_nw_grid<false>(sc, o, d, r[6], keys ? keys[i] : 0ull, t, face, &cnt)
                         : hit_world_nw<false, false>(sc, o, d, r[6], keys ? keys[i] : 0ull, t, face, &cnt);
  out_id[i] = k < 0 ? -1 : k < sc.nobj ? sc.obj_id[k] : sc.med_id[k - sc.nobj];
  out_t[i] = t;
  out_face[i] = face;
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
  DevObj *obj = nullptr;
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
  float4 *nodes = nullptr;  // 2 * nnodes: lo[] then hi[]
  int32_t nobj = 0, nnodes = 0, ninst = 0, nmat = 0, ntex = 0;
  // uniform grid: descriptor, global arrays, brute-force list
  bool grid_ok = false;
  NwGridDesc grid{};
  int32_t grid_max_cell = 0;
  uint16_t *grid_cells = nullptr, *grid_refs = nullptr;
  int32_t *grid_big = nullptr;
  int32_t nbig = 0;
  int32_t accel = RT_NW_ACCEL_AUTO;
  float bg[3] = {0.f, 0.f, 0.f};
  int32_t has_media = 0;
  unsigned long long *accum = nullptr;
  size_t accum_cap = 0;
  float *scratch = nullptr;
  size_t scratch_cap = 0;
  unsigned long long *segments = nullptr;
  unsigned *counter = nullptr;  // persistent kernel's work-item counter
  int32_t persist_blocks = 0;   // resident 16-wave blocks (CUs x blocks per CU), BVH kernels
  int32_t persist_blocks_grid = 0;  // the same for the general grid kernel
  // spheres-only scene (spheres and moving spheres, no instances or media,
  // solid and checker-of-solid textures): the persistent grid kernel's S
  // instantiation, with the other kinds' code compiled out (fewer VGPRs, more
  // waves); RTMI_NW_SIMPLE=0 turns it off (A/B and tests)
  bool simple = false;
  bool simple_ok = !(std::getenv("RTMI_NW_SIMPLE") && std::getenv("RTMI_NW_SIMPLE")[0] == '0');
  int32_t persist_blocks_simple = 0;
  int32_t cus = 0;  // compute units of the device
  // resident blocks per CU of a persistent launch, by (kernel, dynamic LDS
  // bytes): the occupancy query repeated with the bytes the launch stages
  std::vector<std::pair<std::pair<const void *, size_t>, int32_t>> occupancy;
  int32_t last_kernel[4] = {0, 0, 0, 0};  // rt_nw_ctx_last_kernel
  // samples per work item forced by RTMI_NW_CHUNK (A/B only; 0 = automatic),
  // read when the context is created
  int32_t env_chunk = std::getenv("RTMI_NW_CHUNK") ? std::atoi(std::getenv("RTMI_NW_CHUNK")) : 0;
  // the buffers above are shared by every render of the context: a render on
  // another stream first waits for the end of the last one (as rt_ctx)
  hipStream_t last_stream = nullptr;
  hipEvent_t last_done = nullptr;
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
  v.nlo = c->nodes;
  v.nhi = c->nodes + c->nnodes;
  v.nnodes = c->nnodes;
  for (int i = 0; i < 3; ++i) v.bg[i] = c->bg[i];
  v.has_media = c->has_media;
  v.grid = c->grid;
  v.gbig = c->grid_big;
  v.nbig = c->nbig;
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
  HIP_TRY(hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming));
  if (int rc = alloc_copy<unsigned long long>(&ctx->segments, nullptr, 1)) return rc;
  HIP_TRY(hipMemset(ctx->segments, 0, sizeof(unsigned long long)));
  if (int rc = alloc_copy<unsigned>(&ctx->counter, nullptr, 1)) return rc;
  {
    int per_cu = 0;  // the persistent grid: what stays resident (VGPR-limited: one 16-wave block per CU)
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)render_persistent<true, false, false>,
                                                         64 * kPWaves, 0));
    ctx->persist_blocks = per_cu * prop.multiProcessorCount;
    per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)render_persistent<true, true, true>,
                                                         64 * kPWaves, 0));
    ctx->persist_blocks_grid = per_cu * prop.multiProcessorCount;
    per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)render_persistent<true, true, true, true>,
                                                         64 * persist_waves<true>(), 0));
    ctx->persist_blocks_simple = per_cu * prop.multiProcessorCount;
    ctx->cus = prop.multiProcessorCount;
  }
  *out = ctx.release();
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_destroy(rt_nw_ctx *ctx) {
  if (!ctx) return RT_OK;
  Guard g(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (void *p : {(void *)ctx->obj, (void *)ctx->obj_id, (void *)ctx->med, (void *)ctx->med_id, (void *)ctx->inst, (void *)ctx->mat, (void *)ctx->tex,
                  (void *)ctx->pvec, (void *)ctx->pperm, (void *)ctx->img, (void *)ctx->imgd, (void *)ctx->nodes,
                  (void *)ctx->accum, (void *)ctx->scratch, (void *)ctx->segments, (void *)ctx->counter,
                  (void *)ctx->grid_cells, (void *)ctx->grid_refs, (void *)ctx->grid_big})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(ctx->stream);
  if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
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
  // nodes as lo[] = {bmin, skip} and hi[] = {bmax, leaf} (two independent loads)
  std::vector<float4> split(2 * ds.nodes.size());
  for (size_t i = 0; i < ds.nodes.size(); ++i) {
    const Node &nd = ds.nodes[i];
    float sk, lf;
    std::memcpy(&sk, &nd.skip, 4);
    std::memcpy(&lf, &nd.leaf, 4);
    split[i] = make_float4(nd.bmin[0], nd.bmin[1], nd.bmin[2], sk);
    split[ds.nodes.size() + i] = make_float4(nd.bmax[0], nd.bmax[1], nd.bmax[2], lf);
  }
  std::vector<DevObj> dobj(ds.obj.size());
  for (size_t i = 0; i < ds.obj.size(); ++i) {
    const Obj &o = ds.obj[i];
    DevObj &q = dobj[i];
    for (int c = 0; c < 4; ++c) {
      q.g0[c] = o.g0[c];
      q.g1[c] = o.g1[c];
    }
    q.ka = o.kind | (o.aux << 8);
    q.mat = o.mat;
    q.t1 = o.g2[0];
    q.inst = o.inst;
  }
  std::vector<float4> pv(ds.perlin_vec.size() / 4);
  std::memcpy(pv.data(), ds.perlin_vec.data(), pv.size() * sizeof(float4));
  if (ds.grid_ok) {  // (checked before any device buffer is replaced)
    for (uint16_t r : ds.grid_refs)
      if (r >= ds.obj.size()) return set_error(RT_EINVAL, "rt_nw: grid reference out of range");
    for (int32_t b : ds.grid_big)
      if (b < 0 || size_t(b) >= ds.obj.size()) return set_error(RT_EINVAL, "rt_nw: brute-force index out of range");
  }
  Guard g(ctx->device);
  // the context's structures are replaced below: until that completes, no
  // render may use a mix of old counts and new buffers
  ctx->nobj = ctx->nmed = ctx->nnodes = 0;
  ctx->grid_ok = false;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  int rc;
  if ((rc = alloc_copy(&ctx->obj, dobj.data(), dobj.size())) ||
      (rc = alloc_copy(&ctx->med, ds.med.data(), ds.med.size())) ||
      (rc = alloc_copy(&ctx->med_id, ds.med_id.data(), ds.med_id.size())) ||
      (rc = alloc_copy(&ctx->obj_id, ds.obj_id.data(), ds.obj_id.size())) ||
      (rc = alloc_copy(&ctx->inst, ds.inst.data(), ds.inst.size())) ||
      (rc = alloc_copy(&ctx->mat, ds.mat.data(), ds.mat.size())) ||
      (rc = alloc_copy(&ctx->tex, ds.tex.data(), ds.tex.size())) || (rc = alloc_copy(&ctx->pvec, pv.data(), pv.size())) ||
      (rc = alloc_copy(&ctx->pperm, ds.perlin_perm.data(), ds.perlin_perm.size())) ||
      (rc = alloc_copy(&ctx->img, ds.image_px.data(), ds.image_px.size())) ||
      (rc = alloc_copy(&ctx->imgd, ds.image.data(), ds.image.size())) ||
      (rc = alloc_copy(&ctx->nodes, split.data(), split.size())))
    return rc;
  if (ds.grid_ok) {
    if ((rc = alloc_copy(&ctx->grid_cells, ds.grid_cell_start.data(), ds.grid_cell_start.size())) ||
        (rc = alloc_copy(&ctx->grid_refs, ds.grid_refs.data(), ds.grid_refs.size())) ||
        (rc = alloc_copy(&ctx->grid_big, ds.grid_big.data(), ds.grid_big.size())))
      return rc;
    NwGridDesc &G = ctx->grid;
    for (int a = 0; a < 3; ++a) {
      G.g0[a] = ds.grid_g0[a];
      G.h[a] = ds.grid_h[a];
      G.inv_h[a] = ds.grid_inv_h[a];
      G.g1[a] = ds.grid_g1[a];
      G.n[a] = ds.grid_n[a];
    }
    G.ncells = int32_t(ds.grid_cell_start.size()) - 1;
    G.nrefs = int32_t(ds.grid_refs.size());
    G.cell_start = ctx->grid_cells;
    G.refs = ctx->grid_refs;
    ctx->nbig = int32_t(ds.grid_big.size());
    ctx->grid_max_cell = ds.grid_max_cell;
  } else {
    ctx->grid = NwGridDesc{};
    ctx->nbig = 0;
    ctx->grid_max_cell = 0;
  }
  ctx->grid_ok = ds.grid_ok;
  ctx->nobj = int32_t(ds.obj.size());
  ctx->nmed = int32_t(ds.med.size());
  ctx->nnodes = int32_t(ds.nodes.size());
  ctx->ninst = ni;
  ctx->nmat = nm;
  ctx->ntex = nt;
  for (int c = 0; c < 3; ++c) ctx->bg[c] = ds.background[c];
  ctx->has_media = ds.has_media ? 1 : 0;
  bool simple = ds.med.empty();
  for (const Obj &o : ds.obj) simple = simple && o.inst < 0 && (o.kind == kSphere || o.kind == kMovingSphere);
  for (const Tex &t : ds.tex)
    simple = simple && (t.kind == kSolid || (t.kind == kChecker && ds.tex[size_t(t.a)].kind == kSolid &&
                                             ds.tex[size_t(t.b)].kind == kSolid));
  ctx->simple = simple;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_info(rt_nw_ctx *ctx, int32_t *n_prims, int32_t *n_nodes) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (n_prims) *n_prims = ctx->nobj + ctx->nmed;
  if (n_nodes) *n_nodes = ctx->nnodes;
  return RT_OK;
}

namespace {
// The structure a render uses (RT_NW_ACCEL_BVH or _GRID) and whether its
// grid fits the LDS of the persistent / grid kernel shapes.
constexpr int32_t kNwGridMaxCell = 24;  // AUTO: a grid with a fuller cell renders with the BVH
size_t grid_bytes(const rt_nw_ctx *c) {
  return nw_grid_lds_bytes(c->nobj, c->grid.ncells, c->grid.nrefs, c->nbig);
}
int32_t accel_used(const rt_nw_ctx *c) {
  // the grid is staged whole: by the persistent kernel (one block per CU)
  // when it runs, else by the grid kernel's per-block budget; a grid that
  // fits neither renders with the BVH
  const bool persist = RTMI_NW_PERSIST && c->persist_blocks_grid > 0;
  const bool fits = c->grid_ok && grid_bytes(c) <= (persist ? kPLdsBudget : kLdsBudget);
  if (c->accel == RT_NW_ACCEL_GRID) return fits ? RT_NW_ACCEL_GRID : RT_NW_ACCEL_BVH;
  if (c->accel == RT_NW_ACCEL_BVH) return RT_NW_ACCEL_BVH;
  return fits && c->grid_max_cell <= kNwGridMaxCell ? RT_NW_ACCEL_GRID : RT_NW_ACCEL_BVH;
}
}  // namespace

RTMI_EXPORT int rt_nw_ctx_set_accel(rt_nw_ctx *ctx, int32_t accel) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (accel != RT_NW_ACCEL_AUTO && accel != RT_NW_ACCEL_BVH && accel != RT_NW_ACCEL_GRID)
    return set_error(RT_EINVAL, "rt_nw_ctx_set_accel: unknown structure %d", accel);
  ctx->accel = accel;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_ctx_accel_info(rt_nw_ctx *ctx, int32_t *accel, int32_t *dims3, int32_t *max_cell, int32_t *n_big) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (accel) *accel = accel_used(ctx);
  if (dims3)
    for (int a = 0; a < 3; ++a) dims3[a] = ctx->grid_ok ? ctx->grid.n[a] : 0;
  if (max_cell) *max_cell = ctx->grid_ok ? ctx->grid_max_cell : 0;
  if (n_big) *n_big = ctx->grid_ok ? ctx->nbig : 0;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_render_rows(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t spp,
                                  int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows,
                                  float *dev_strip, void *stream) {
  if (!ctx || !cam || !dev_strip) return set_error(RT_EINVAL, "rt_nw_render_rows: null argument");
  if (ctx->nobj + ctx->nmed <= 0) return set_error(RT_EINVAL, "no scene uploaded (rt_nw_ctx_set_scene)");
  if (W < 1 || H < 1 || spp < 1 || spp >= (1 << 24) || max_depth < 1 || max_depth >= (1 << 24) ||
      int64_t(W) * H >= (int64_t(1) << 40))
    return set_error(RT_EINVAL, "rt_nw_render_rows: bad size (W, H, spp >= 1, spp < 2^24, 1 <= max_depth < 2^24)");
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
  // kernel shape: persistent when the nodes fit one CU's LDS budget, else grid
  const size_t node_bytes = size_t(ctx->nnodes) * 32, obj_bytes = size_t(ctx->nobj) * (sizeof(DevObj) + 4);
  const bool use_grid = accel_used(ctx) == RT_NW_ACCEL_GRID;
  const size_t gbytes = use_grid ? grid_bytes(ctx) : 0;
  const bool persist = RTMI_NW_PERSIST && (use_grid ? ctx->persist_blocks_grid > 0 : ctx->persist_blocks > 0) &&
                       (use_grid || (ctx->nnodes > 0 && node_bytes <= kPLdsBudget));
  // the spheres-only instantiation of the persistent grid kernel
  const bool simple = persist && use_grid && ctx->simple && ctx->simple_ok && ctx->persist_blocks_simple > 0;
  const int32_t pblocks = simple ? ctx->persist_blocks_simple : use_grid ? ctx->persist_blocks_grid : ctx->persist_blocks;
  const int64_t pwaves = simple ? persist_waves<true>() : kPWaves;
  // samples per work item (same image for any size; RTMI_NW_CHUNK overrides,
  // for A/B).  Persistent kernel: ~80 items per resident wave, 4..32 samples:
  // the final scene (fog, lights: long and uneven paths) at 256 spp runs 329
  // ms with 8, 433 with 32; at 1024 spp 1215 ms with 24, 1205 with 32, 1308
  // with 8 — the item count, not the size, sets its tail
  // (profiles/r01/session6/nw_chunk.txt).  Grid kernel: 32.
  // (samples per work item: set below, once the resident grid is known)
  // the context's buffers (accumulator, counters) are shared by every render:
  // a render on another stream first waits for the last one
  if (ctx->last_stream && ctx->last_stream != st) HIP_TRY(hipStreamWaitEvent(st, ctx->last_done, 0));
  ctx->last_stream = st;
  struct MarkDone {  // record the end of this render's work, whatever path returns
    rt_nw_ctx *c;
    hipStream_t s;
    ~MarkDone() { (void)hipEventRecord(c->last_done, s); }
  } mark_done{ctx, st};
  if (valid < nrows)  // rows past H: zero
    HIP_TRY(hipMemsetAsync(dev_strip + size_t(valid) * W * 3, 0, size_t(nrows - valid) * W * 3 * sizeof(float), st));
  HIP_TRY(hipMemsetAsync(ctx->segments, 0, sizeof(unsigned long long), st));
  const View v = view_of(ctx);
  // objects staged beside the nodes only when two blocks still fit a CU (or
  // when one block per CU is all the nodes allow anyway)
  const bool p_objs = RTMI_NW_LDS_OBJS && persist &&
                      (node_bytes + obj_bytes <= kPTwoBlockBudget ||
                       (node_bytes > kPTwoBlockBudget && node_bytes + obj_bytes <= kPLdsBudget));
  const bool g_grid = use_grid && !persist && gbytes <= kLdsBudget;  // grid kernel with the grid staged per block
  if (use_grid && !persist && !g_grid) return set_error(RT_EINVAL, "rt_nw: grid does not fit the grid kernel's LDS");
  const bool lds_nodes = !persist && !use_grid && ctx->nnodes > 0 && node_bytes <= kLdsBudget,
             lds_objs = RTMI_NW_LDS_OBJS && lds_nodes && node_bytes + obj_bytes <= kLdsBudget;
  const size_t lds = use_grid ? gbytes
                     : persist ? (p_objs ? node_bytes + obj_bytes : node_bytes)
                               : lds_objs ? node_bytes + obj_bytes : lds_nodes ? node_bytes : 0;
  // the kernel that will run, its static LDS beside the staged bytes, and
  // (persistent) how many of its blocks stay resident with those bytes
  const void *kfn = simple ? (const void *)render_persistent<true, true, true, true>
                    : persist && use_grid ? (const void *)render_persistent<true, true, true>
                    : persist && p_objs ? (const void *)render_persistent<true, true, false>
                    : persist ? (const void *)render_persistent<true, false, false>
                    : g_grid ? (const void *)render_kernel<true, false, false, true>
                    : lds_objs ? (const void *)render_kernel<true, true, true, false>
                    : lds_nodes ? (const void *)render_kernel<true, true, false, false>
                                : (const void *)render_kernel<true, false, false, false>;
  {
    hipFuncAttributes fa;
    HIP_TRY(hipFuncGetAttributes(&fa, kfn));
    if (fa.sharedSizeBytes + lds > kCuLds)
      return set_error(RT_EINVAL, "rt_nw: %zu B staged + %zu B static LDS exceed a CU's %zu B", lds,
                       size_t(fa.sharedSizeBytes), kCuLds);
  }
  int32_t resident = pblocks;
  if (persist) {
    const auto key = std::make_pair(kfn, lds);
    auto it = std::find_if(ctx->occupancy.begin(), ctx->occupancy.end(), [&](const auto &e) { return e.first == key; });
    if (it == ctx->occupancy.end()) {
      int per_cu = 0;
      HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, int(64 * pwaves), lds));
      ctx->occupancy.push_back({key, std::max(1, per_cu) * ctx->cus});
      it = ctx->occupancy.end() - 1;
    }
    resident = it->second;
  }
  int64_t chunk = 32;
  if (persist) {
    const int64_t waves = int64_t(resident) * pwaves;
    chunk = std::min<int64_t>(32, std::max<int64_t>(4, int64_t(a.tiles) * spp / (80 * waves)));
  }
  // (at most 65535 samples per item: job indices stay below 2^22, where the
  // kernels' reciprocal-multiply job decode is exact)
  a.chunk = std::min<int64_t>({spp, ctx->env_chunk > 0 ? ctx->env_chunk : chunk, 65535});
  a.nch = (spp + a.chunk - 1) / a.chunk;
  if (int64_t(a.tiles) * a.nch >= (int64_t(1) << 31) - kWaves) return set_error(RT_EINVAL, "render too large");
  a.n_items = a.tiles * a.nch;
  const unsigned blocks = persist ? unsigned(std::min<int64_t>(resident, (a.n_items + pwaves - 1) / pwaves))
                                  : unsigned((a.n_items + kWaves - 1) / kWaves);
  if (persist) HIP_TRY(hipMemsetAsync(ctx->counter, 0, sizeof(unsigned), st));
  ctx->last_kernel[0] = persist ? 1 : 0;
  ctx->last_kernel[1] = use_grid ? 1 : 0;
  ctx->last_kernel[2] = simple ? 1 : 0;
  ctx->last_kernel[3] = a.chunk;
  auto launch = [&](auto chunked) {
    constexpr bool C = decltype(chunked)::value;
    if (simple)
      hipLaunchKernelGGL((render_persistent<C, true, true, true>), dim3(blocks), dim3(64 * persist_waves<true>()), lds, st, v, a, ctx->accum, dev_strip, ctx->segments, ctx->counter);
    else if (persist && use_grid)
      hipLaunchKernelGGL((render_persistent<C, true, true>), dim3(blocks), dim3(64 * kPWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments, ctx->counter);
    else if (persist && p_objs)
      hipLaunchKernelGGL((render_persistent<C, true, false>), dim3(blocks), dim3(64 * kPWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments, ctx->counter);
    else if (persist)
      hipLaunchKernelGGL((render_persistent<C, false, false>), dim3(blocks), dim3(64 * kPWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments, ctx->counter);
    else if (g_grid)
      hipLaunchKernelGGL((render_kernel<C, false, false, true>), dim3(blocks), dim3(64 * kWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments);
    else if (lds_objs)
      hipLaunchKernelGGL((render_kernel<C, true, true, false>), dim3(blocks), dim3(64 * kWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments);
    else if (lds_nodes)
      hipLaunchKernelGGL((render_kernel<C, true, false, false>), dim3(blocks), dim3(64 * kWaves), lds, st, v, a, ctx->accum, dev_strip, ctx->segments);
    else
      hipLaunchKernelGGL((render_kernel<C, false, false, false>), dim3(blocks), dim3(64 * kWaves), 0, st, v, a, ctx->accum, dev_strip, ctx->segments);
  };
  if (a.nch > 1) {
    const size_t nv = size_t(valid) * W * 3;
    if (nv > ctx->accum_cap) {
      HIP_TRY(hipStreamSynchronize(st));
      if (int rc = alloc_copy<unsigned long long>(&ctx->accum, nullptr, nv)) return rc;
      ctx->accum_cap = nv;
    }
    HIP_TRY(hipMemsetAsync(ctx->accum, 0, nv * sizeof(unsigned long long), st));
    launch(std::true_type{});
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(finalize_kernel, dim3(unsigned((nv + 255) / 256)), dim3(256), 0, st, ctx->accum, dev_strip, nv);
  } else {
    launch(std::false_type{});
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

RTMI_EXPORT int rt_nw_debug_trace(rt_nw_ctx *ctx, const rt_nw_camera *cam, int32_t W, int32_t H, int32_t max_depth,
                                  uint64_t seed, int32_t i, int32_t j, int32_t s, float *rec, int32_t cap, int32_t *n) {
  if (!ctx || !cam || !rec || !n || cap < 1 || max_depth < 1 || i < 0 || i >= W || j < 0 || j >= H)
    return set_error(RT_EINVAL, "rt_nw_debug_trace: bad argument");
  Guard g(ctx->device);
  Args a{};
  a.cam = camf(cam->cam);
  a.time0 = float(cam->time0);
  a.time1 = float(cam->time1);
  a.W = W;
  a.H = H;
  a.max_depth = max_depth;
  a.seed = seed;
  float *d_rec = nullptr;
  int *d_n = nullptr;
  HIP_TRY(hipMalloc(&d_rec, size_t(cap) * 12 * sizeof(float)));
  HIP_TRY(hipMalloc(&d_n, sizeof(int)));
  hipLaunchKernelGGL(trace_kernel, dim3(1), dim3(64), 0, ctx->stream, view_of(ctx), a, i, j, s, d_rec, cap, d_n);
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(n, d_n, sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(rec, d_rec, size_t(*n) * 12 * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(d_rec);
  (void)hipFree(d_n);
  if (e != hipSuccess) return set_error(RT_EHIP, "rt_nw_debug_trace: %s", hipGetErrorString(e));
  return RT_OK;
}

RTMI_EXPORT int rt_nw_debug_hits(rt_nw_ctx *ctx, const float *rays, const uint64_t *keys, int32_t n, int32_t *out_id,
                                 float *out_t, int32_t *out_face) {
  if (!ctx || (n > 0 && (!rays || !out_id || !out_t || !out_face)) || n < 0)
    return set_error(RT_EINVAL, "rt_nw_debug_hits: bad argument");
  if (ctx->nobj + ctx->nmed <= 0) return set_error(RT_EINVAL, "no scene uploaded (rt_nw_ctx_set_scene)");
  if (n == 0) return RT_OK;
  Guard g(ctx->device);
  const bool grid = accel_used(ctx) == RT_NW_ACCEL_GRID;
  const size_t lds = grid ? grid_bytes(ctx) : 0;
  if (lds > kCuLds) return set_error(RT_EUNSUPPORTED, "rt_nw_debug_hits: grid of %zu B exceeds a CU's LDS", lds);
  float *d_rays = nullptr, *d_t = nullptr;
  unsigned long long *d_keys = nullptr;
  int32_t *d_id = nullptr, *d_face = nullptr;
  hipError_t e = hipMalloc(&d_rays, size_t(n) * 8 * sizeof(float));
  if (e == hipSuccess && keys) e = hipMalloc(&d_keys, size_t(n) * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc(&d_t, size_t(n) * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&d_id, size_t(n) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&d_face, size_t(n) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(d_rays, rays, size_t(n) * 8 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && keys) e = hipMemcpy(d_keys, keys, size_t(n) * sizeof(unsigned long long), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const dim3 grd(unsigned((n + 255) / 256)), blk(256);
    if (grid)
      hipLaunchKernelGGL(debug_hits_kernel<true>, grd, blk, lds, ctx->stream, view_of(ctx), d_rays, d_keys, n, d_id,
                         d_t, d_face);
    else
      hipLaunchKernelGGL(debug_hits_kernel<false>, grd, blk, 0, ctx->stream, view_of(ctx), d_rays, d_keys, n, d_id,
                         d_t, d_face);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out_id, d_id, size_t(n) * sizeof(int32_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(out_t, d_t, size_t(n) * sizeof(float), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(out_face, d_face, size_t(n) * sizeof(int32_t), hipMemcpyDeviceToHost);
  (void)hipFree(d_rays);
  (void)hipFree(d_keys);
  (void)hipFree(d_t);
  (void)hipFree(d_id);
  (void)hipFree(d_face);
  if (e != hipSuccess) return set_error(RT_EHIP, "rt_nw_debug_hits: %s", hipGetErrorString(e));
  return RT_OK;
}

// Analysis builds only (RTMI_NW_PHASES): the phase cycle sums since the last
// call (see g_nw_phase), zeroed after reading; RT_EUNSUPPORTED otherwise.
// RTMI_STATS build (librtmi_stats.so): the executed-work counters of the
// launches since the last call (see g_nw_stats), zeroed after reading;
// RT_EUNSUPPORTED in the product build.
RTMI_EXPORT int rt_nw_debug_counters(uint64_t *out4) {
#if RTMI_STATS
  if (!out4) return set_error(RT_EINVAL, "null");
  HIP_TRY(hipDeviceSynchronize());
  unsigned long long v[4] = {0, 0, 0, 0}, z[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_nw_stats), sizeof v));
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_nw_stats), z, sizeof z));
  for (int q = 0; q < 4; ++q) out4[q] = v[q];
  return RT_OK;
#else
  (void)out4;
  return set_error(RT_EUNSUPPORTED, "rt_nw_debug_counters: not an RTMI_STATS build");
#endif
}

RTMI_EXPORT int rt_nw_debug_phases(uint64_t *out4) {
#if RTMI_NW_PHASES
  if (!out4) return set_error(RT_EINVAL, "null");
  HIP_TRY(hipDeviceSynchronize());
  unsigned long long v[4];
  HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_nw_phase), sizeof v));
  for (int q = 0; q < 4; ++q) out4[q] = v[q];
  const unsigned long long z[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_nw_phase), z, sizeof z));
  return RT_OK;
#else
  (void)out4;
  return set_error(RT_EUNSUPPORTED, "rt_nw_debug_phases: not an RTMI_NW_PHASES build");
#endif
}

RTMI_EXPORT int rt_nw_ctx_last_kernel(rt_nw_ctx *ctx, int32_t *out4) {
  if (!ctx || !out4) return set_error(RT_EINVAL, "null");
  for (int q = 0; q < 4; ++q) out4[q] = ctx->last_kernel[q];
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
