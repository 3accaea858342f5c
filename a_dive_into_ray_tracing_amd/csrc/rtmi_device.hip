// rtmi_device.hip — device half of librtmi.so: the gfx950 path-tracing
// kernels and the C-ABI entry points that launch them.
//
// Hot path: the per-pixel sample loop of the
// reference — camera ray (camera.h:56-62), the iterative ray_color bounce
// loop (main.cpp:57-83), hittable_list::hit / sphere::hit (hittable_list.h:
// 20-34, sphere.h:21-55), lambertian/metal/dielectric scatter (material.h),
// RNG (rtweekend.h:21-29) and the per-pixel sum (main.cpp:276-285).
//
// MI355X design:
//  * One wavefront owns a work item = (64-pixel tile, range of samples).
//    Lanes take (pixel, sample) jobs from a wave-local queue: when a lane's
//    path terminates, __ballot + mbcnt hand it the next job (path
//    regeneration with wavefront prefix compaction), so lanes stay busy until
//    the item's last samples and never wait for the slowest pixel.
//  * The sphere loop is wave-uniform: sphere k's {centre, r^2} is one
//    s_load_dwordx4 into SGPRs for the whole wave (scalar cache, 16 B per
//    sphere), so the VALU does only the ray-sphere arithmetic.
//  * Counter-based RNG (xoroshiro128+ seeded per (seed, pixel, sample)) and
//    int64 fixed-point accumulation (LDS ds_add_u64, then one global atomic
//    per pixel per item) make the image independent of scheduling, tiling,
//    partition and GPU count, and bit-identical to the CPU restatement
//    (oracle/, fast mode).
//  * No MFMA: this is branchy scalar FP32 (VALU roofline).
//
// Numerics: compiled with -ffp-contract=off; every FMA is an explicit
// __builtin_fma(f); division and sqrt are IEEE correctly rounded (hipcc
// default).  The DOUBLE instantiation (FAST=false) reproduces the reference
// bit-for-bit given its rand() stream (rt_replay_worker).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rtmi_internal.h"
#include "rtmi_path.h"


namespace rtmi {

// ---------------------------------------------------------------------------
// fast render kernel
// ---------------------------------------------------------------------------
struct RenderArgs {
  Cam<float> cam;
  int32_t n, npairs, W, H, spp, max_depth;
  uint64_t seed;
  int32_t row0, row_step, nrows_valid;
  int32_t tiles_x, n_items;
  // two-phase schedule: phase 1 = samples [0, spp1) in
  // chunks of chunk1, phase 2 = [spp1, spp) in chunks of chunk2; phase-2 items
  // come last in the grid, so the dispatch tail is one short item
  int32_t tiles, spp1, chunk1, nch1, chunk2, nch2;
  // grid kernel: every block's items share one tile (nch1 a multiple of the
  // block's waves, no phase 2), so the block sums its waves' accumulators and
  // flushes once (a quarter of the global atomics)
  int32_t block_flush;
  // block_flush launches whose block covers ALL samples of its tile (items
  // per tile == waves per block, not a progressive pass): the block writes the
  // tile's float sums straight to the output strip — no accumulator memset,
  // global atomics or finalize pass (config 2: 500 spp = 4 items of 125)
  int32_t block_owns_tile;
  // the fixed-point accumulators' byte offset in the dynamic LDS (past the
  // acceleration structure; launch_tw)
  int32_t acc_off;
  // progressive passes: this launch renders samples s_base + [0, spp)
  int32_t s_base;
  uint64_t out_elems;  // elements of accum / out (RTMI_CHECK builds verify every write)
  Accel acc;           // BVH kernels only
  // cost-ordered dispatch: tile rank -> tile (null: identity)
  // and per-tile world.hit counts of this launch (null: not measured)
  const int32_t *tile_order;
  unsigned *tile_cost;
};

#ifndef RTMI_WAVES_PER_BLOCK
#define RTMI_WAVES_PER_BLOCK 4
#endif
constexpr int kWavesPerBlock = RTMI_WAVES_PER_BLOCK;
#ifndef RTMI_WAVES_PER_EU
#define RTMI_WAVES_PER_EU 1
#endif
// RTMI_TRACE builds record one line per wave (analysis only): start/end
// (s_memrealtime, 100 MHz), CU id and items taken, world.hit calls.
#ifndef RTMI_TRACE
#define RTMI_TRACE 0
#endif
#if RTMI_TRACE
constexpr unsigned kTraceCap = 1u << 18;
__device__ unsigned long long g_trace[kTraceCap * 4];
__device__ unsigned g_trace_n;
#define RTMI_TRACE_BEGIN                                                                 \
  const unsigned long long trace_t0 = __builtin_amdgcn_s_memrealtime();                  \
  const unsigned long long cyc_start = __builtin_amdgcn_s_memtime();
#define RTMI_TRACE_END(items, wsegs)                                                     \
  if (lane == 0) {                                                                       \
    atomicAdd(&segments[5], cnt.cyc_hit);                                                \
    atomicAdd(&segments[6], __builtin_amdgcn_s_memtime() - cyc_start);                   \
    const unsigned k_ = atomicAdd(&g_trace_n, 1u);                                       \
    if (k_ < kTraceCap) {                                                                \
      g_trace[4 * k_] = trace_t0;                                                        \
      g_trace[4 * k_ + 1] = __builtin_amdgcn_s_memrealtime();                            \
      g_trace[4 * k_ + 2] = (uint64_t(__builtin_amdgcn_s_getreg(0xF804)) << 32) |        \
                            uint64_t(unsigned(items));                                   \
      g_trace[4 * k_ + 3] = (uint64_t(blockIdx.x * (blockDim.x >> 6) + wave) << 32) |     \
                            (uint64_t(wsegs) & 0xFFFFFFFFull);                           \
    }                                                                                    \
  }
#else
#define RTMI_TRACE_BEGIN
#define RTMI_TRACE_END(items, wsegs)
#endif

// RTMI_CHECK builds (analysis only) bounds-check every accumulator write and
// count violations in segments[5..7] instead of performing them.
#ifndef RTMI_CHECK
#define RTMI_CHECK 0
#endif
#ifndef RTMI_PERSIST_MIN_BLOCKS
#define RTMI_PERSIST_MIN_BLOCKS 1
#endif
#ifndef RTMI_SYNC_PROBE
#define RTMI_SYNC_PROBE 0
#endif
// The experimental build (make experimental -> lib/librtmi_experimental.so):
// the resident grid kernel (RT_KERNEL_RESIDENT), measured
// slower than render_kernel — kept and tested, out of the product library,
// where RT_KERNEL_RESIDENT runs the automatic choice.  (The queue kernel of
// round 5, RT_KERNEL_QUEUE, was retired in round 6: 33-44% slower and a ring
// stall in ~2% of renders; git show 1b6ce15:a_dive_into_ray_tracing_amd/csrc/rtmi_device.hip)
#ifndef RTMI_EXPERIMENTAL
#define RTMI_EXPERIMENTAL 0
#endif
#ifndef RTMI_PAIR_GROUP
#define RTMI_PAIR_GROUP 4
#endif
constexpr int kPairGroup = RTMI_PAIR_GROUP;  // sphere pairs per scalar-load group

// Per-sample colour -> int64 fixed point (2^-32).  Guarded: NaN -> 0 and
// the value clamped to [0, 64], so the conversion is always defined and a
// sum of up to 2^24 samples cannot overflow (64 * 2^24 * 2^32 = 2^62);
// every scene here stays far inside (RTIOW colours are <= 1).  The oracle
// applies the identical guard.
// q / d for 0 <= q < 2^22 and 1 <= d <= 2^16, given inv_d = 1.0f / d: the
// float quotient is within one of the true one, fixed by one correction.
__device__ __forceinline__ int div_small(int q, int d, float inv_d) {
  int t = int(float(q) * inv_d);
  const int r = q - t * d;
  t += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
  return t;
}

// a wave-uniform float pinned to a scalar register
__device__ __forceinline__ float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

__device__ __forceinline__ int64_t to_fixed(float c) {
  // branch-free: v_med3 clamps to [0, 64] (inf included), NaN selects 0; then
  // trunc(g * 2^32) as two 32-bit halves (g >= 0: trunc = floor): the
  // integer part, and the fraction (exact) scaled by 2^32 (exact, < 2^32) —
  // 8 VALU instead of the 64-bit conversion's 15
  const float g = c == c ? __builtin_amdgcn_fmed3f(c, 0.0f, 64.0f) : 0.0f;
  const uint32_t hi = uint32_t(g);
  const uint32_t lo = uint32_t((g - float(hi)) * 4294967296.0f);
  return int64_t((uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ float from_fixed(int64_t v) { return float(v) * 0x1p-32f; }

// Grid-kernel block shape.  A block holds its wave slots (and LDS) until its
// slowest wave ends, so big blocks fragment the CU: with 8-wave blocks the
// per-wave trace shows ~6 500 of 8 192 wave slots resident in steady state.
// The BVH kernel runs 4-wave blocks at 8 waves per SIMD (64 VGPRs, a few
// spilled): 16-byte nodes and 16-bit leaf indices keep a block's LDS (BVH +
// accumulators) under 20 KB, so 8 blocks fit a CU.  Config 2: 16-wave blocks
// 55.2 ms, 8-wave 52.4, 4-wave (7 per CU, int32 indices) 51.9.  The
// brute-force loop keeps its own shape (kWavesPerBlock).
#ifndef RTMI_BVH_WAVES
#define RTMI_BVH_WAVES 4
#endif
#ifndef RTMI_ACC_PER_EU
#define RTMI_ACC_PER_EU 8
#endif
template <bool BVH> struct GridShape {
  static constexpr int waves = BVH ? RTMI_BVH_WAVES : kWavesPerBlock;
  static constexpr int per_eu = BVH ? RTMI_ACC_PER_EU : RTMI_WAVES_PER_EU;
};
// The persistent kernel runs brute-force scenes only: with the BVH or the
// grid it measured slower than the grid kernel everywhere (round 2: config 2
// frame / 1/8 strip 30.9 / 4.72 ms against 26.0 / 3.70; profiles/README.md),
// so RT_KERNEL_PERSISTENT with an accelerator runs the grid kernel.  (The
// CU-resident designs of rounds 5-6 are DESIGN.md §4.6-4.7.)

// The camera and the reciprocals of main.cpp:278-279's (W-1, H-1)
// denominators in LDS (21 floats), read at each regeneration instead of held
// in scalar registers (config 2: 30.1 -> 28.2 ms: the scalar registers the
// camera occupied were spilled to VGPR lanes and read back with v_readlane).
// Fast mode: u, v = (i + ju) * (1/(W-1)), (j + jv) * (1/(H-1)) — <= 1 ulp from
// the reference's quotients, two divisions fewer per camera ray (the
// oracle's fast mode computes the same products).
__device__ __forceinline__ void stage_camera(float *cam_lds, const RenderArgs &a) {
  const unsigned t = threadIdx.x;
  if (t < 19) {
    float v;
    switch (t / 3) {
      case 0: v = (&a.cam.origin.x)[t % 3]; break;
      case 1: v = (&a.cam.llc.x)[t % 3]; break;
      case 2: v = (&a.cam.hor.x)[t % 3]; break;
      case 3: v = (&a.cam.ver.x)[t % 3]; break;
      case 4: v = (&a.cam.u.x)[t % 3]; break;
      case 5: v = (&a.cam.v.x)[t % 3]; break;
      default: v = a.cam.lens; break;
    }
    cam_lds[t] = v;
  } else if (t < 21) {
    cam_lds[t] = 1.0f / float((t == 19 ? a.W : a.H) - 1);
  }
}
__device__ __forceinline__ Cam<float> lds_camera(const float *cam_lds) {
  Cam<float> cm;
  cm.origin = mk(cam_lds[0], cam_lds[1], cam_lds[2]);
  cm.llc = mk(cam_lds[3], cam_lds[4], cam_lds[5]);
  cm.hor = mk(cam_lds[6], cam_lds[7], cam_lds[8]);
  cm.ver = mk(cam_lds[9], cam_lds[10], cam_lds[11]);
  cm.u = mk(cam_lds[12], cam_lds[13], cam_lds[14]);
  cm.v = mk(cam_lds[15], cam_lds[16], cam_lds[17]);
  cm.lens = cam_lds[18];
  return cm;
}
// Per-lane work counters of the analysis builds (RTMI_STATS: the executed
// work; RTMI_TRACE_PHASES / RTMI_TRACE: cycle clocks); empty in the product.
struct SegCounters {
#if RTMI_STATS
  unsigned stats[4];      // brute force: groups, groups with a candidate (wave), resolves (lane), sphere resolves (wave)
  unsigned bvh_stats[5];  // BVH / grid: node (cell) visits, leaf (cell) sphere tests (lane); node iterations,
                          // leaf-sphere iterations, root resolutions (wave)
#endif
#if RTMI_TRACE_PHASES
  PhaseClock pc;
#endif
#if RTMI_TRACE
  unsigned long long cyc_hit;
#endif
};

__device__ __forceinline__ void flush_counters(const SegCounters &cnt, int lane, unsigned long long *segments) {
#if RTMI_STATS
  // brute force: [1] groups, [2] groups with a candidate, [4] sphere
  // resolves (wave); BVH / grid: [1] node iterations, [2] leaf-sphere
  // iterations, [4] root resolutions (wave).  [3] resolves (lane), [5] node
  // visits, [6] leaf sphere tests (lane).
  if (lane == 0) {
    atomicAdd(&segments[1], (unsigned long long)cnt.stats[0]);
    atomicAdd(&segments[2], (unsigned long long)cnt.stats[1]);
    atomicAdd(&segments[4], (unsigned long long)cnt.stats[3]);
  }
  atomicAdd(&segments[3], (unsigned long long)cnt.stats[2]);
  atomicAdd(&segments[5], (unsigned long long)cnt.bvh_stats[0]);
  atomicAdd(&segments[6], (unsigned long long)cnt.bvh_stats[1]);
  atomicAdd(&segments[1], (unsigned long long)cnt.bvh_stats[2]);
  atomicAdd(&segments[2], (unsigned long long)cnt.bvh_stats[3]);
  atomicAdd(&segments[4], (unsigned long long)cnt.bvh_stats[4]);
#else
  (void)cnt, (void)lane, (void)segments;
#endif
}

// Closest-hit kinds of the accelerated kernels (template ACC): 1 BVH, 2 the
// uniform grid in LDS, 3 the same walked as one y layer, 4 / 5 the grid (one
// layer) walked in global memory (a grid over the LDS budget)
constexpr bool acc_grid(int A) { return A >= 2; }
constexpr bool acc_flat(int A) { return A == 3 || A == 5; }
constexpr bool acc_gmem(int A) { return A >= 4; }

// One segment of a path — the body of the reference's recursive ray_color
// (main.cpp:57-83) as one step of an iterative loop: the closest hit (brute
// force, BVH or grid: the same hit bit for bit), then the sky of a miss,
// absorption, or the scattered ray with its robustness offset.  Returns true
// when the path ended: col is then its colour (black when absorbed or out of
// depth).  Shared by every fast kernel, so they compute identical paths.
template <int ACC>
__device__ __forceinline__ bool path_segment(const SceneView<float> &sc, const SpherePair *__restrict__ pairs,
                                             const RenderArgs &a, V3<float> &o, V3<float> &d, V3<float> &T,
                                             int &depth, Xoro &rng, V3<float> &col, SegCounters &cnt,
                                             unsigned long long *segments) {
  (void)cnt, (void)segments;
  float t;
#if RTMI_TRACE
  const unsigned long long cyc0 = __builtin_amdgcn_s_memtime();
#endif
  int k;
  uint32_t key = 0u;  // the grid's hit slot (hit_world_grid)
  if constexpr (ACC == 1) {
    k = hit_world_bvh<kBigGroup>(a.acc, o, d, t
#if RTMI_STATS
                                  , cnt.bvh_stats
#endif
    );
  } else if constexpr (ACC >= 2) {
    k = hit_world_grid<kBigGroup, acc_flat(ACC), acc_gmem(ACC)>(a.acc, o, d, t, key
#if RTMI_STATS
                                   , cnt.bvh_stats
#endif
#if RTMI_TRACE_PHASES
                                   , cnt.pc
#endif
                                   );
  } else {
    k = hit_world_packed<kPairGroup>(pairs, a.npairs, o, d, t
#if RTMI_STATS
                                     , cnt.stats
#endif
    );
  }
#if RTMI_TRACE
  cnt.cyc_hit += __builtin_amdgcn_s_memtime() - cyc0;
#endif
#if RTMI_CHECK
  if (k >= a.n) atomicAdd(&segments[7], 1ull << 32);
#endif
  // 1/|d| once for the lanes that need it: the sky of a miss (main.cpp:80)
  // and unit(din) of metal and dielectric — the same expression
  const bool miss = k < 0 || (RTMI_CHECK && k >= a.n);
  // the hit sphere's three records in one memory round trip (a miss reads
  // sphere 0's, unused)
  const int kk = miss ? 0 : k;
  // the grid kernels hold the hit sphere's {c, S} in LDS at the hit's record
  // slot (stage_grid): the hit record's geometry from there, one global
  // gather fewer (19.82 -> 19.73 ms, profiles/r03/ab_geom_lds.txt)
  const float4 sh1k = sc.sh1[kk], sh0k = sc.sh0[kk];
  float4 geomk;
  if constexpr (acc_gmem(ACC)) geomk = *reinterpret_cast<const float4 *>(a.acc.grid_gmem + key);
  else geomk = ACC >= 2 ? lds_sphere(key) : sc.geom[kk];
  const int kind = miss ? -1 : int(sh1k.x);
  float inv_len = 0.0f;
  if (kind != RT_MAT_LAMBERTIAN) inv_len = drcp(dsqrt(dot<true>(d, d)));
  if (miss) {
    const V3<float> sk = sky_fast(d, inv_len);
    col = mk(T.x * sk.x, T.y * sk.y, T.z * sk.z);
    return true;
  }
  V3<float> p, nrm, at, nd;
  bool front;
  hit_record_fast(geomk, sh0k.x, o, d, t, p, nrm, front);
  if (!scatter_fast(sh0k, sh1k, d, nrm, front, rng, at, nd, inv_len))
    return true;  // absorbed (metal below the surface): black, main.cpp:78
  T = mk(T.x * at.x, T.y * at.y, T.z * at.z);
  // float robustness: start the next segment
  // 2^-14 * (1 + |p|_inf) off the surface, on the side the scattered ray
  // leaves on, so float hit-point error (~1e-6) cannot re-hit the surface
  // just left or trap the path inside an opaque sphere.
  float m = __builtin_fabsf(p.x);
  if (__builtin_fabsf(p.y) > m) m = __builtin_fabsf(p.y);
  if (__builtin_fabsf(p.z) > m) m = __builtin_fabsf(p.z);
  float delta = 0x1p-14f * (1.0f + m);
  if (dot<true>(nd, nrm) < 0.f) delta = -delta;
  o = mk(__builtin_fmaf(delta, nrm.x, p.x), __builtin_fmaf(delta, nrm.y, p.y), __builtin_fmaf(delta, nrm.z, p.z));
  d = nd;
  // depth exhausted: black, main.cpp:58-60 (the depth is the low 24 bits:
  // render_kernel keeps the path's pixel above them)
  return (++depth & 0xFFFFFF) >= a.max_depth;
}

// ACC: 0 brute force, 1 BVH, 2 uniform grid (RT_ACCEL_*), 3 the grid walked as one
// y layer (hit_world_grid<.., true>); the accelerated
// kernels stage their structure in LDS and share the block shape.
template <int TW, bool CHUNKED, int ACC>
__global__ __launch_bounds__(64 * GridShape<ACC != 0>::waves, GridShape<ACC != 0>::per_eu) void render_kernel(
    const float4 *__restrict__ geom, const float4 *__restrict__ sh0, const float4 *__restrict__ sh1,
    const SpherePair *__restrict__ pairs, RenderArgs a, unsigned long long *__restrict__ accum,
    float *__restrict__ out, unsigned long long *__restrict__ segments) {
  constexpr int TH = 64 / TW;
  constexpr int WPB = GridShape<ACC != 0>::waves;
  __shared__ float cam_lds[21];  // the camera (stage_camera)
  __shared__ unsigned blk_seg[WPB];  // the waves' world.hit counts (block_flush)
#if RTMI_SYNC_PROBE
  __shared__ int blk_any[2];
  if (threadIdx.x < 2) blk_any[threadIdx.x] = 0;  // (published by the staging barrier)
#endif
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * WPB + wave;
  // The per-pixel int64 fixed-point sums, in the dynamic LDS past the
  // acceleration structure: one set per wave, or (block_flush: the block's
  // waves share one tile) one set the four waves add into together — integer
  // sums, so the same bits in any order, and 4.5 KB less LDS per block, which
  // keeps 8 blocks per CU with the grid's record slots (grid_lds_bytes).
  // Zeroed before the staging barrier, which publishes it.
  const bool acc_shared = CHUNKED && a.block_flush;
  unsigned long long *const acc_lds =
      reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(rtmi_bvh_lds) + a.acc_off);
  for (int i = threadIdx.x; i < (acc_shared ? 3 * 64 : WPB * 3 * 64); i += 64 * WPB) acc_lds[i] = 0;
  unsigned long long *const acc = acc_lds + (acc_shared ? 0 : wave * 3 * 64);  // [3][64]
  stage_camera(cam_lds, a);
  if constexpr (ACC == 0) __syncthreads();  // (accelerated kernels: stage_* ends with one)
  if constexpr (ACC == 1) stage_bvh(a.acc);  // block barrier inside: before any wave leaves
  else if constexpr (acc_gmem(ACC)) stage_grid_desc(a.acc);
  else if constexpr (ACC >= 2) stage_grid(a.acc);
#if RTMI_SYNC_PROBE
  const bool has_item = item < a.n_items;  // every wave stays for the per-pass block barriers
#else
  if (item >= a.n_items) return;  // wave-uniform; no block barrier follows
  constexpr bool has_item = true;
#endif

  auto item_range = [&](int it, int &tl, int &sb, int &n) {
    if (it < a.tiles * a.nch1) {
      tl = it / a.nch1;
      sb = (it - tl * a.nch1) * a.chunk1;
      n = max(0, min(a.chunk1, a.spp1 - sb));  // 0: an empty item of the automatic schedule
    } else {
      const int i2 = it - a.tiles * a.nch1;
      tl = i2 / a.nch2;
      sb = a.spp1 + (i2 - tl * a.nch2) * a.chunk2;
      n = max(0, min(a.chunk2, a.spp - sb));
    }
  };
  int tile, s0, ns;
  item_range(has_item ? item : 0, tile, s0, ns);
  if (!has_item) ns = 0;
  if (a.tile_order) tile = a.tile_order[tile];  // expensive tiles first
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int x0 = tx * TW, y0 = ty * TH;
  const int vw = min(TW, a.W - x0), vh = min(TH, a.nrows_valid - y0);
  const int nv = vw * vh;  // valid pixels of this tile
  const int nq = nv * ns;  // jobs: (pixel, sample) pairs of this item

  unsigned nseg = 0;  // world.hit calls of this wave (wave-uniform; algorithmic-work accounting)
  RTMI_TRACE_BEGIN
  SegCounters cnt{};
#if RTMI_TRACE_PHASES
  unsigned long long cyc_iter = 0, cyc_regen = 0, cyc_ramp = 0;
#endif

  const SceneView<float> sc{geom, sh0, sh1, a.n};

  V3<float> o, d, T;
  // the path's pixel in the tile (bits 24..29) and its depth (bits 0..23;
  // max_depth < 2^24, check_render_args) in one register
  int pxd = 0;
  bool active = true;
  Xoro rng;

  // job q -> pixel px = q % nv, sample s0 + q / nv (sample-major, so every
  // pixel of the tile advances together); then the camera ray.
  // q / d = umulhi(2q, ceil(2^31 / d)), exact for 1 <= d <= 64 and q < 2^25
  // (the error q (m d - 2^31) / (d 2^31) < q / 2^31 stays below 1/d; job
  // indices are < 2^22); the multipliers are wave-uniform integers (scalar
  // registers)
  const uint32_t m_nv = 0x7FFFFFFFu / uint32_t(max(nv, 1)) + 1u, m_vw = 0x7FFFFFFFu / uint32_t(vw) + 1u;
  auto camera_ray = [&](int q, V3<float> &ro, V3<float> &rd, Xoro &g) {
    const int qs = int(__umulhi(uint32_t(q) << 1, m_nv));
    const int s = s0 + qs;
    const int p = q - qs * nv;
    const int ly = int(__umulhi(uint32_t(p) << 1, m_vw)), lx = p - ly * vw;
    const int i = x0 + lx;
    const int j = a.row0 + (y0 + ly) * a.row_step;
    g.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(a.s_base + s));
    float ju, jv;
    g.pair(ju, jv);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // camera read here, not hoisted out of the loop
    const float u = (float(i) + ju) * cam_lds[19];  // main.cpp:278, by the reciprocal
    const float v = (float(j) + jv) * cam_lds[20];  // main.cpp:279
    get_ray<true, float>(lds_camera(cam_lds), u, v, g, ro, rd);
  };
  // a lane takes job q with its camera ray (or goes idle when the item has
  // no job q)
  auto adopt = [&](int q, const V3<float> &ro, const V3<float> &rd, const Xoro &g) {
    if (q < nq) {
      o = ro;
      d = rd;
      rng = g;
      pxd = (q - int(__umulhi(uint32_t(q) << 1, m_nv)) * nv) << 24;
      T = mk(1.f, 1.f, 1.f);
    } else {
      active = false;
    }
  };

  // Camera-ray pool: lane L holds the camera ray of job
  // pbase + L, generated by all 64 lanes at once; a lane whose path ended
  // takes the next unused slot through ds_bpermute.  The ray generation runs
  // with every lane busy, once per 64 jobs, instead of once per loop pass
  // for the few lanes that regenerate.  Same rays bit for bit.
  V3<float> po, pd;
  Xoro prng;
  int pbase = 0, ppos = 64;  // wave-uniform: job of slot 0, next unused slot
  camera_ray(lane, po, pd, prng);
  adopt(lane, po, pd, prng);
  auto pull = [](int src4, float v) { return __int_as_float(__builtin_amdgcn_ds_bpermute(src4, __float_as_int(v))); };
  auto pull64 = [](int src4, uint64_t v) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_ds_bpermute(src4, int(uint32_t(v))));
    const uint32_t hi = uint32_t(__builtin_amdgcn_ds_bpermute(src4, int(uint32_t(v >> 32))));
    return (uint64_t(hi) << 32) | lo;
  };

#if RTMI_SYNC_PROBE
  // Analysis only (RTMI_SYNC_PROBE=1): the block's waves pass in lockstep, two
  // block barriers per pass, until none of them has a live path — the
  // synchronisation a block-level regrouping of rays would need (DESIGN.md
  // §8.2), without the regrouping.  block_flush launches only (every wave of
  // the block has an item).
  for (int pass = 0;; ++pass) {
    const unsigned long long live = __ballot(active);
    if (lane == 0 && live) atomicOr(&blk_any[pass & 1], 1);
    __syncthreads();
    const int any_live = blk_any[pass & 1];
    __syncthreads();
    if (threadIdx.x == 0) blk_any[pass & 1] = 0;  // reused two passes on, after two more barriers
    if (!any_live) break;
    if (live == 0) continue;
#else
  for (;;) {
    const unsigned long long live = __ballot(active);
    if (live == 0) break;
#endif
    nseg = unsigned(__builtin_amdgcn_readfirstlane(int(nseg + unsigned(__popcll(live)))));
    bool done = false;
    V3<float> col = mk(0.f, 0.f, 0.f);
#if RTMI_TRACE_PHASES
    const unsigned long long cyc_a = __builtin_amdgcn_s_memtime();
#endif
    if (active) {
      done = path_segment<ACC>(sc, pairs, a, o, d, T, pxd, rng, col, cnt, segments);
    }
#if RTMI_TRACE_PHASES
    const unsigned long long cyc_b = __builtin_amdgcn_s_memtime();
    cyc_iter += cyc_b - cyc_a;  // hit + shading of this pass (wave-level)
    const bool ramp = pbase + ppos >= nq;  // the item's jobs all handed out: the wave's ramp-down
#endif
    const unsigned long long m = __ballot(done);
    if (m) {
      if (done) {
        const int px = pxd >> 24;
        atomicAdd(&acc[px], (unsigned long long)to_fixed(col.x));
        atomicAdd(&acc[64 + px], (unsigned long long)to_fixed(col.y));
        atomicAdd(&acc[128 + px], (unsigned long long)to_fixed(col.z));
      }
      const int rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
      // ranks [0, cnt) take slots ppos, ppos + 1, ...: at most two rounds,
      // the second after a refill for the next 64 jobs (skipped once the
      // item has none: those lanes go idle)
      const int cnt = __popcll(m);
      for (int served = 0; served < cnt;) {
        if (ppos == 64) {
          pbase = __builtin_amdgcn_readfirstlane(pbase + 64);
          ppos = 0;
          if (pbase < nq) camera_ray(pbase + lane, po, pd, prng);
        }
        const int take = min(cnt - served, 64 - ppos);
        const int r = rank - served;
        const int src4 = ((ppos + r) & 63) << 2;  // every lane reads (ds_bpermute reads active lanes only)
        V3<float> ro, rd;
        Xoro g;
        ro = mk(pull(src4, po.x), pull(src4, po.y), pull(src4, po.z));
        rd = mk(pull(src4, pd.x), pull(src4, pd.y), pull(src4, pd.z));
        g.s0 = pull64(src4, prng.s0);
        g.s1 = pull64(src4, prng.s1);
        if (done && r >= 0 && r < take) adopt(pbase + ppos + r, ro, rd, g);
        ppos = __builtin_amdgcn_readfirstlane(ppos + take);
        served = __builtin_amdgcn_readfirstlane(served + take);
      }
    }
#if RTMI_TRACE_PHASES
    const unsigned long long cyc_e = __builtin_amdgcn_s_memtime();
    cyc_regen += cyc_e - cyc_b;
    if (ramp) cyc_ramp += cyc_e - cyc_a;
#endif
  }

  // world.hit count and tile cost: per wave, or (block_flush: the block's
  // waves share the tile) summed in LDS and added once per block at the
  // flush — 30 000 instead of 120 000 single-lane global atomics at config 2
  const bool block_counts = CHUNKED && a.block_flush;
  if (lane == 0) {
    if (block_counts) {
      blk_seg[wave] = nseg;
    } else {
      atomicAdd(segments, (unsigned long long)nseg);
      if (a.tile_cost) atomicAdd(&a.tile_cost[tile], nseg);
    }
  }
  flush_counters(cnt, lane, segments);
#if RTMI_TRACE_PHASES
  // [1] big spheres + clip/setup, [2] loop passes after the item's last job
  // was taken (ramp-down), [3] cell walk
  cnt.pc.c[0] += cnt.pc.c[1];
  cnt.pc.c[1] = cyc_ramp;
  if (lane == 0) for (int q = 0; q < 3; ++q) atomicAdd(&segments[1 + q], cnt.pc.c[q]);
  // wave-level: [4] hit + shading passes, [7] accumulation + regeneration
  if (lane == 0) { atomicAdd(&segments[4], cyc_iter); atomicAdd(&segments[7], cyc_regen); }
#endif
  RTMI_TRACE_END(1, nseg)
  // the lane index recomputed here, not kept live (in scratch) since the
  // accumulator's initialisation
  int fl = int(threadIdx.x & 63u);
  asm volatile("" : "+v"(fl));
  if constexpr (CHUNKED) {
    if (a.block_flush) {  // block-uniform; no wave of this block returned early
      __syncthreads();
      if (block_counts && threadIdx.x == 0) {
        unsigned bseg = 0;
#pragma unroll
        for (int w = 0; w < WPB; ++w) bseg += blk_seg[w];
        atomicAdd(segments, (unsigned long long)bseg);
        if (a.tile_cost) atomicAdd(&a.tile_cost[tile], bseg);
      }
      if (wave == 0 && fl < nv) {
        const int ly = fl / vw, lx = fl - ly * vw;
        const size_t o3 = (size_t(y0 + ly) * size_t(a.W) + size_t(x0 + lx)) * 3;
        for (int c = 0; c < 3; ++c) {
          const unsigned long long v = acc[64 * c + fl];  // (acc_shared: the block's sums)
          if (a.block_owns_tile) out[o3 + c] = from_fixed((long long)v);
          else atomicAdd(&accum[o3 + c], v);
        }
      }
      return;
    }
  }
  if (fl < nv && has_item) {
    const int ly = fl / vw, lx = fl - ly * vw;
    const size_t o3 = (size_t(y0 + ly) * size_t(a.W) + size_t(x0 + lx)) * 3;
#if RTMI_CHECK
    if (o3 + 3 > a.out_elems) {
      atomicAdd(&segments[5], 1ull);
      atomicMax(&segments[6], (unsigned long long)o3);
    } else
#endif
    for (int c = 0; c < 3; ++c) {
      const unsigned long long v = acc[64 * c + fl];
      if constexpr (CHUNKED) atomicAdd(&accum[o3 + c], v);
      else out[o3 + c] = from_fixed((long long)v);
    }
  }
}

#if RTMI_EXPERIMENTAL
// ---------------------------------------------------------------------------
// resident grid kernel (RT_KERNEL_RESIDENT; experimental
// build only: measured 3% slower than render_kernel, profiles/r06/resident/)
// ---------------------------------------------------------------------------
// render_kernel's per-wave loop in CU-resident blocks: each wave takes work
// items from a global counter until none is left, with its own fixed-point
// sums in LDS, flushed (global atomics, or the floats when the item covers
// all samples of its tile) at the end of every item.  No wave waits for
// another: render_kernel's 4-wave block holds its wave slots until its
// slowest wave ends, and a launch drains as those blocks do (one rank's 1/8
// strip of config 2: 86-93% of the 8 192 wave slots resident mid-run, the
// slots emptying over the last ~30% of the launch).  Here every
// slot stays busy until the counter runs out, and the tail is each wave's
// last item.  Blocks of kResWaves waves stage the structure once (two copies
// per CU instead of eight).  Same per-path arithmetic (path_segment) and
// integer sums: the image is bit-identical to every other kernel's.
#ifndef RTMI_RES_WAVES
#define RTMI_RES_WAVES 16
#endif
constexpr int kResWaves = RTMI_RES_WAVES;
static_assert(kResWaves >= 1 && kResWaves <= 16, "a block holds at most 16 waves");

template <int TW, int ACC>
__global__ __launch_bounds__(64 * kResWaves, 8) void render_resident(
    const float4 *__restrict__ geom, const float4 *__restrict__ sh0, const float4 *__restrict__ sh1,
    RenderArgs a, unsigned long long *__restrict__ accum, float *__restrict__ out,
    unsigned long long *__restrict__ segments, unsigned *__restrict__ counter) {
  static_assert(ACC >= 1, "accelerated scenes only (brute force: render_persistent)");
  constexpr int TH = 64 / TW;
  __shared__ float cam_lds[21];  // the camera (stage_camera)
  // The arguments the item decode and the flush read, in LDS: read there
  // once per item instead of held in scalar registers through the path
  // loop (held, they spilled 45 scalar registers into VGPR lanes and 2-14
  // VGPRs to scratch)
  enum { kTiles, kNch1, kChunk1, kSpp1, kNch2, kChunk2, kSpp, kTilesX, kW, kRows, kNItems, kOwns, kFirst,
         kOrder, kCost = kOrder + 2, kAccum = kCost + 2, kOut = kAccum + 2, kCounter = kOut + 2,
         kSegs = kCounter + 2, kArgs = kSegs + 2 };
  __shared__ uint32_t args_lds[kArgs];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    const int32_t v[kFirst + 1] = {a.tiles, a.nch1, a.chunk1, a.spp1, a.nch2, a.chunk2, a.spp, a.tiles_x, a.W,
                                   a.nrows_valid, a.n_items, a.block_owns_tile, int32_t(gridDim.x) * kResWaves};
    for (int i = 0; i <= kFirst; ++i) args_lds[i] = uint32_t(v[i]);
    auto ptr = [&](int at, const void *p) {
      args_lds[at] = uint32_t(size_t(p));
      args_lds[at + 1] = uint32_t(size_t(p) >> 32);
    };
    ptr(kOrder, a.tile_order);
    ptr(kCost, a.tile_cost);
    ptr(kAccum, accum);
    ptr(kOut, out);
    ptr(kCounter, counter);
    ptr(kSegs, segments);
  }
  // (read after a workgroup fence, so not hoisted out of the item loop)
  auto arg = [&](int i) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return int(__builtin_amdgcn_readfirstlane(int(args_lds[i])));
  };
  auto arg_ptr = [&](int i) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(args_lds[i])));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(args_lds[i + 1])));
    return reinterpret_cast<void *>((size_t(hi) << 32) | lo);
  };
  // this wave's sums [3][64], in the dynamic LDS past the structure; zeroed
  // before the staging barrier, which publishes them, and again by every flush
  unsigned long long *const acc =
      reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(rtmi_bvh_lds) + a.acc_off) + wave * 3 * 64;
  for (int c = 0; c < 3; ++c) acc[64 * c + lane] = 0;
  stage_camera(cam_lds, a);
  if constexpr (ACC == 1) stage_bvh(a.acc);  // (each ends with the block barrier)
  else if constexpr (acc_gmem(ACC)) stage_grid_desc(a.acc);
  else stage_grid(a.acc);

  const SceneView<float> sc{geom, sh0, sh1, a.n};
  SegCounters cnt{};
  RTMI_TRACE_BEGIN
#if RTMI_TRACE
  unsigned wsegs = 0;
  int items_done = 0;
#endif
  auto pull = [](int src4, float v) { return __int_as_float(__builtin_amdgcn_ds_bpermute(src4, __float_as_int(v))); };
  auto pull64 = [](int src4, uint64_t v) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_ds_bpermute(src4, int(uint32_t(v))));
    const uint32_t hi = uint32_t(__builtin_amdgcn_ds_bpermute(src4, int(uint32_t(v >> 32))));
    return (uint64_t(hi) << 32) | lo;
  };
  // the first item by position, the next ones from the counter (which the
  // host zeroes: items past the grid's first gridDim.x * kResWaves)
  int item = blockIdx.x * kResWaves + wave;
  while (item < arg(kNItems)) {
    int tile, s0, ns;
    {
      const int tiles = arg(kTiles), nch1 = arg(kNch1), chunk1 = arg(kChunk1);
      if (item < tiles * nch1) {
        tile = item / nch1;
        s0 = (item - tile * nch1) * chunk1;
        ns = max(0, min(chunk1, arg(kSpp1) - s0));
      } else {
        const int nch2 = arg(kNch2), chunk2 = arg(kChunk2);
        const int i2 = item - tiles * nch1;
        tile = i2 / nch2;
        s0 = arg(kSpp1) + (i2 - tile * nch2) * chunk2;
        ns = max(0, min(chunk2, arg(kSpp) - s0));
      }
      const int32_t *order = static_cast<const int32_t *>(arg_ptr(kOrder));
      if (order) tile = order[tile];  // expensive tiles first
    }
    tile = __builtin_amdgcn_readfirstlane(tile);
    const int tiles_x = arg(kTilesX);
    const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const int x0 = tx * TW, y0 = ty * TH;
    const int vw = min(TW, a.W - x0), vh = min(TH, arg(kRows) - y0);
    const int nv = vw * vh;
    const int nq = nv * ns;
    unsigned nseg = 0;

    // the per-wave loop of render_kernel (path regeneration from the
    // camera-ray pool; see there)
    V3<float> o, d, T;
    int pxd = 0;
    bool active = true;
    Xoro rng;
    const uint32_t m_nv = 0x7FFFFFFFu / uint32_t(max(nv, 1)) + 1u, m_vw = 0x7FFFFFFFu / uint32_t(vw) + 1u;
    auto camera_ray = [&](int q, V3<float> &ro, V3<float> &rd, Xoro &g) {
      const int qs = int(__umulhi(uint32_t(q) << 1, m_nv));
      const int s = s0 + qs;
      const int p = q - qs * nv;
      const int ly = int(__umulhi(uint32_t(p) << 1, m_vw)), lx = p - ly * vw;
      const int i = x0 + lx;
      const int j = a.row0 + (y0 + ly) * a.row_step;
      g.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(a.s_base + s));
      float ju, jv;
      g.pair(ju, jv);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // camera read here, not hoisted out of the loop
      const float u = (float(i) + ju) * cam_lds[19];  // main.cpp:278, by the reciprocal
      const float v = (float(j) + jv) * cam_lds[20];  // main.cpp:279
      get_ray<true, float>(lds_camera(cam_lds), u, v, g, ro, rd);
    };
    auto adopt = [&](int q, const V3<float> &ro, const V3<float> &rd, const Xoro &g) {
      if (q < nq) {
        o = ro;
        d = rd;
        rng = g;
        pxd = (q - int(__umulhi(uint32_t(q) << 1, m_nv)) * nv) << 24;
        T = mk(1.f, 1.f, 1.f);
      } else {
        active = false;
      }
    };
    V3<float> po, pd;
    Xoro prng;
    int pbase = 0, ppos = 64;
    camera_ray(lane, po, pd, prng);
    adopt(lane, po, pd, prng);
    for (;;) {
      const unsigned long long live = __ballot(active);
      if (live == 0) break;
      nseg = unsigned(__builtin_amdgcn_readfirstlane(int(nseg + unsigned(__popcll(live)))));
      bool done = false;
      V3<float> col = mk(0.f, 0.f, 0.f);
      if (active) done = path_segment<ACC>(sc, nullptr, a, o, d, T, pxd, rng, col, cnt, segments);
      const unsigned long long m = __ballot(done);
      if (m) {
        if (done) {
          const int px = pxd >> 24;
          atomicAdd(&acc[px], (unsigned long long)to_fixed(col.x));
          atomicAdd(&acc[64 + px], (unsigned long long)to_fixed(col.y));
          atomicAdd(&acc[128 + px], (unsigned long long)to_fixed(col.z));
        }
        const int rank = __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u));
        const int cnt_done = __popcll(m);
        for (int served = 0; served < cnt_done;) {
          if (ppos == 64) {
            pbase = __builtin_amdgcn_readfirstlane(pbase + 64);
            ppos = 0;
            if (pbase < nq) camera_ray(pbase + lane, po, pd, prng);
          }
          const int take = min(cnt_done - served, 64 - ppos);
          const int r = rank - served;
          const int src4 = ((ppos + r) & 63) << 2;
          V3<float> ro, rd;
          Xoro g;
          ro = mk(pull(src4, po.x), pull(src4, po.y), pull(src4, po.z));
          rd = mk(pull(src4, pd.x), pull(src4, pd.y), pull(src4, pd.z));
          g.s0 = pull64(src4, prng.s0);
          g.s1 = pull64(src4, prng.s1);
          if (done && r >= 0 && r < take) adopt(pbase + ppos + r, ro, rd, g);
          ppos = __builtin_amdgcn_readfirstlane(ppos + take);
          served = __builtin_amdgcn_readfirstlane(served + take);
        }
      }
    }
    // the next item's claim first: its latency overlaps the flush
    unsigned next = 0;
    if (lane == 0) {
      next = atomicAdd(static_cast<unsigned *>(arg_ptr(kCounter)), 1u);
      atomicAdd(static_cast<unsigned long long *>(arg_ptr(kSegs)), (unsigned long long)nseg);
      unsigned *const cost = static_cast<unsigned *>(arg_ptr(kCost));
      if (cost) atomicAdd(&cost[tile], nseg);
    }
#if RTMI_TRACE
    wsegs += nseg;
    ++items_done;
#endif
    // flush: the item's sums (the lane index recomputed, not kept live)
    int fl = int(threadIdx.x & 63u);
    asm volatile("" : "+v"(fl));
    if (fl < nv) {
      const int ly = fl / vw, lx = fl - ly * vw;
      const size_t o3 = (size_t(y0 + ly) * size_t(arg(kW)) + size_t(x0 + lx)) * 3;
#if RTMI_CHECK
      if (o3 + 3 > a.out_elems) {
        atomicAdd(&segments[5], 1ull);
        atomicMax(&segments[6], (unsigned long long)o3);
      } else
#endif
      if (arg(kOwns)) {
        float *const o = static_cast<float *>(arg_ptr(kOut));
        for (int c = 0; c < 3; ++c) o[o3 + c] = from_fixed((long long)acc[64 * c + fl]);
      } else {
        unsigned long long *const g = static_cast<unsigned long long *>(arg_ptr(kAccum));
        for (int c = 0; c < 3; ++c) atomicAdd(&g[o3 + c], acc[64 * c + fl]);
      }
    }
    for (int c = 0; c < 3; ++c) acc[64 * c + fl] = 0;
    item = arg(kFirst) + __builtin_amdgcn_readfirstlane(int(next));
  }
  flush_counters(cnt, lane, segments);
  RTMI_TRACE_END(items_done, wsegs)
}
#endif  // RTMI_EXPERIMENTAL

// ---------------------------------------------------------------------------
// persistent render kernel: continuous per-wave job stream over work items
// ---------------------------------------------------------------------------
// A fixed grid of waves pulls work items (tile, sample range) from a global
// counter.  A wave holds two items at a time in two LDS accumulator slots:
// lanes take jobs from the current item; when it has no jobs left the wave
// fetches the next item into the other slot and keeps its lanes busy, while
// the paths of the previous item finish; that slot is flushed (one global
// atomic per pixel and channel) as soon as none of its paths is in flight.
// So no lane waits for the slowest path of an item, and the grid's tail is a
// few paths long.  Same per-path arithmetic as render_kernel (bit-identical).
struct ItemDesc {
  int x0, y0, vw, nv, s0, nq, tile;
};

template <int TW>
__device__ __forceinline__ ItemDesc describe_item(const RenderArgs &a, int item) {
  constexpr int TH = 64 / TW;
  int tile, s0, ns;
  if (item < a.tiles * a.nch1) {
    tile = item / a.nch1;
    s0 = (item - tile * a.nch1) * a.chunk1;
    ns = max(0, min(a.chunk1, a.spp1 - s0));
  } else {
    const int i2 = item - a.tiles * a.nch1;
    tile = i2 / a.nch2;
    s0 = a.spp1 + (i2 - tile * a.nch2) * a.chunk2;
    ns = max(0, min(a.chunk2, a.spp - s0));
  }
  if (a.tile_order) tile = a.tile_order[tile];  // expensive tiles first
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  ItemDesc r;
  r.x0 = tx * TW;
  r.y0 = ty * TH;
  r.vw = min(TW, a.W - r.x0);
  const int vh = min(TH, a.nrows_valid - r.y0);
  r.nv = r.vw * vh;
  r.s0 = s0;
  r.nq = r.nv * ns;
  r.tile = tile;
  return r;
}

template <int TW, bool CHUNKED>
__global__ __launch_bounds__(64 * kWavesPerBlock, RTMI_PERSIST_MIN_BLOCKS) void render_persistent(
    const float4 *__restrict__ geom, const float4 *__restrict__ sh0, const float4 *__restrict__ sh1,
    const SpherePair *__restrict__ pairs, RenderArgs a, unsigned long long *__restrict__ accum,
    float *__restrict__ out, unsigned long long *__restrict__ segments, unsigned *__restrict__ counter) {
  constexpr int WPB = kWavesPerBlock;
  __shared__ unsigned long long acc[WPB][2][3][64];
  __shared__ unsigned long long wave_segs[WPB];
  __shared__ unsigned slot_segs[WPB][2];  // world.hit calls of each slot's item (tile cost)
  // each slot's item: x0, y0, vw, nv, s_base + s0, tile, 1/nv, 1/vw (float
  // bits), read at regeneration and flush: the wave's registers hold only
  // the current item's job counters
  __shared__ int item_lds[WPB][2][8];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ float cam_lds[21];
  stage_camera(cam_lds, a);
  __syncthreads();
  if (lane < 2) slot_segs[wave][lane] = 0;
  for (int s = 0; s < 2; ++s)
    for (int c = 0; c < 3; ++c) acc[wave][s][c][lane] = 0;
  if (lane == 0) wave_segs[wave] = 0;
  unsigned nseg = 0;
  int n_taken = 0;
  RTMI_TRACE_BEGIN
  SegCounters cnt{};
  const SceneView<float> sc{geom, sh0, sh1, a.n};

  // issue-priority rotation, starting at the hardware wave slot
  unsigned prio_phase = __builtin_amdgcn_s_getreg(0xF804) & 15u;
  // wave-uniform slot state: the current item (slot `cur`) hands out jobs;
  // the previous one (slot cur^1, all jobs handed out) may still have paths
  // in flight.
  int cur = 0;
  bool cur_valid = false, prev_valid = false, exhausted = false;
  int cur_next = 0, cur_nq = 0;

  // per-lane path state; px = pixel of the tile | slot << 6
  V3<float> o, d, T;
  int px = 0, depth = 0;
  bool active = false;
  Xoro rng;

  auto flush = [&](int s) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int x0 = item_lds[wave][s][0], y0 = item_lds[wave][s][1], vw = item_lds[wave][s][2];
    if (lane < item_lds[wave][s][3]) {
      const int ly = lane / vw, lx = lane - ly * vw;
      const size_t o3 = (size_t(y0 + ly) * size_t(a.W) + size_t(x0 + lx)) * 3;
#if RTMI_CHECK
      if (o3 + 3 > a.out_elems || s < 0 || s > 1) {
        atomicAdd(&segments[5], 1ull);
        atomicMax(&segments[6], (unsigned long long)o3);
      } else
#endif
      for (int c = 0; c < 3; ++c) {
        const unsigned long long v = acc[wave][s][c][lane];
        if constexpr (CHUNKED) atomicAdd(&accum[o3 + c], v);
        else out[o3 + c] = from_fixed((long long)v);
      }
    }
    for (int c = 0; c < 3; ++c) acc[wave][s][c][lane] = 0;
    if (lane == 0) {
      if (a.tile_cost) atomicAdd(&a.tile_cost[item_lds[wave][s][5]], slot_segs[wave][s]);
      slot_segs[wave][s] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  };

  for (;;) {
    // 1. hand jobs to idle lanes, fetching items as the current one runs dry
    unsigned long long idle = __ballot(!active);
    while (idle) {
      if (cur_valid && cur_next < cur_nq) {
        const int avail = cur_nq - cur_next;
        const int rank = __builtin_amdgcn_mbcnt_hi(unsigned(idle >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(idle), 0u));
        if (((idle >> lane) & 1ull) && rank < avail) {
          // job q -> pixel q % nv, sample s0 + q / nv; then the camera ray
          // (q < nq <= 64 * 65535 < 2^22: div_small is exact, host-checked)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // item and camera read here
          const int *it = item_lds[wave][cur];
          const int nv = it[3], vw = it[2];
          const int q = cur_next + rank;
          const int qs = div_small(q, nv, __int_as_float(it[6]));
          const int p = q - qs * nv;
          const int ly = div_small(p, vw, __int_as_float(it[7])), lx = p - ly * vw;
          const int i = it[0] + lx;
          const int j = a.row0 + (it[1] + ly) * a.row_step;
          rng.init(a.seed, uint64_t(j) * uint64_t(a.W) + uint64_t(i), uint32_t(it[4] + qs));
          float ju, jv;
          rng.pair(ju, jv);
          const float u = (float(i) + ju) * cam_lds[19];  // main.cpp:278, by the reciprocal
          const float v = (float(j) + jv) * cam_lds[20];  // main.cpp:279
          get_ray<true, float>(lds_camera(cam_lds), u, v, rng, o, d);
          T = mk(1.f, 1.f, 1.f);
          depth = 0;
          px = p | (cur << 6);
          active = true;
        }
        cur_next += min(__popcll(idle), avail);
        idle = __ballot(!active);
      } else {
        if (prev_valid || exhausted) break;  // wait for the previous item to drain
        unsigned itn = 0;
        if (lane == 0) itn = atomicAdd(counter, 1u);
        itn = __shfl(itn, 0);
        if (int(itn) >= a.n_items) {
          exhausted = true;
          break;
        }
        ++n_taken;
        prev_valid = cur_valid;  // all its jobs are handed out
        cur ^= 1;
        const ItemDesc cd = describe_item<TW>(a, int(itn));
        if (lane < 8) {
          const int f[8] = {cd.x0, cd.y0, cd.vw, cd.nv, a.s_base + cd.s0, cd.tile,
                            __float_as_int(1.0f / float(max(cd.nv, 1))), __float_as_int(1.0f / float(cd.vw))};
          int v = f[0];
#pragma unroll
          for (int k = 1; k < 8; ++k) v = lane == k ? f[k] : v;
          item_lds[wave][cur][lane] = v;
        }
        cur_nq = cd.nq;
        cur_valid = true;
        cur_next = 0;
      }
    }
    const unsigned long long live = __ballot(active);
    if (live == 0) break;
    {  // world.hit calls per slot (the tiles' cost map)
      const unsigned long long live_cur = __ballot(active && (px >> 6) == cur);
      if (lane == 0) {
        if (live_cur) atomicAdd(&slot_segs[wave][cur], unsigned(__popcll(live_cur)));
        if (live != live_cur) atomicAdd(&slot_segs[wave][cur ^ 1], unsigned(__popcll(live & ~live_cur)));
      }
    }
    // The SIMD issues the oldest ready wave first: in a resident grid the
    // youngest wave of a SIMD gets ~1/10 of the oldest one's issue slots and
    // is left holding items alone at the end.  Rotating the issue priority
    // every segment step gives every wave the same share.
    switch ((prio_phase++) & 3) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }

    // 2. one segment of every live path
    bool done = false;
    V3<float> col = mk(0.f, 0.f, 0.f);
    if (active) {
      ++nseg;
      done = path_segment<0>(sc, pairs, a, o, d, T, depth, rng, col, cnt, segments);
    }
    // 3. finished paths add their colour to their item's slot
#if RTMI_CHECK
    if (done && (px < 0 || px > 127)) {
      atomicAdd(&segments[7], 1ull);
      done = false;
      active = false;
    }
#endif
    if (done) {
      const int s = px >> 6, p = px & 63;
      atomicAdd(&acc[wave][s][0][p], (unsigned long long)to_fixed(col.x));
      atomicAdd(&acc[wave][s][1][p], (unsigned long long)to_fixed(col.y));
      atomicAdd(&acc[wave][s][2][p], (unsigned long long)to_fixed(col.z));
      active = false;
    }
    // 4. flush items whose jobs are all handed out and whose paths are all done
    if (prev_valid && __ballot(active && (px >> 6) != cur) == 0) {
      flush(cur ^ 1);
      prev_valid = false;
    }
    if (cur_valid && cur_next >= cur_nq && __ballot(active && (px >> 6) == cur) == 0) {
      flush(cur);
      cur_valid = false;
    }
  }
  if (prev_valid) flush(cur ^ 1);
  if (cur_valid) flush(cur);

  atomicAdd(&wave_segs[wave], (unsigned long long)nseg);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) atomicAdd(segments, wave_segs[wave]);
  flush_counters(cnt, lane, segments);
  RTMI_TRACE_END(n_taken, wave_segs[wave])
  (void)n_taken;
}


// Closest hit of n given rays by the brute-force loop and by the BVH
// (validation: rt_ctx_debug_hits).  rays = {o.xyz, d.xyz} per ray.
template <int ACC>
__global__ __launch_bounds__(256) void debug_hit_kernel(const SpherePair *__restrict__ pairs, int32_t npairs, Accel acc,
                                                       const float *__restrict__ rays, int32_t n,
                                                       int32_t *__restrict__ out_idx, float *__restrict__ out_t) {
  if constexpr (ACC == 1) stage_bvh(acc);
  else if constexpr (acc_gmem(ACC)) stage_grid_desc(acc);
  else stage_grid(acc);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3<float> o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
  const V3<float> d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
  float t0, t1;
  uint32_t key;
#if RTMI_STATS
  unsigned st[4] = {0, 0, 0, 0}, bst[5] = {0, 0, 0, 0, 0};
  out_idx[2 * i] = hit_world_packed<kPairGroup>(pairs, npairs, o, d, t0, st);
  out_idx[2 * i + 1] = ACC == 1 ? hit_world_bvh<kBigGroup>(acc, o, d, t1, bst) : hit_world_grid<kBigGroup, acc_flat(ACC), acc_gmem(ACC)>(acc, o, d, t1, key, bst);
#else
  out_idx[2 * i] = hit_world_packed<kPairGroup>(pairs, npairs, o, d, t0);
#if RTMI_TRACE_PHASES
  PhaseClock pc{{0, 0, 0}};
  out_idx[2 * i + 1] = ACC == 1 ? hit_world_bvh<kBigGroup>(acc, o, d, t1) : hit_world_grid<kBigGroup, acc_flat(ACC), acc_gmem(ACC)>(acc, o, d, t1, key, pc);
#else
  out_idx[2 * i + 1] = ACC == 1 ? hit_world_bvh<kBigGroup>(acc, o, d, t1) : hit_world_grid<kBigGroup, acc_flat(ACC), acc_gmem(ACC)>(acc, o, d, t1, key);
#endif
#endif
  out_t[2 * i] = t0;
  out_t[2 * i + 1] = t1;
}

__global__ void finalize_kernel(const unsigned long long *__restrict__ accum, float *__restrict__ out, size_t n) {
  const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = from_fixed((long long)accum[i]);
}

// ---------------------------------------------------------------------------
// exact replay kernel (double, reference op order, supplied rand() stream)
// ---------------------------------------------------------------------------
constexpr int kMaxReplayDepth = 64;

struct ReplayArgs {
  Cam<double> cam;
  int32_t n, W, H, spp, max_depth, n_jobs;
};

// ray_color main.cpp:57-83 with the recursion's product order: the colour is
// attenuation_1 * (attenuation_2 * (... * sky)), combined innermost first.
__device__ V3<double> ray_color_exact(const SceneView<double> &sc, V3<double> o, V3<double> d, int max_depth,
                                      StreamRng &g) {
  V3<double> att[kMaxReplayDepth];
  int n_att = 0;
  V3<double> col = mk(0.0, 0.0, 0.0);
  for (int depth = max_depth; depth > 0; depth--) {
    double t;
    const int k = hit_world<false, double>(sc, o, d, t);
    if (k < 0) {
      col = sky<false, double>(d);
      break;
    }
    V3<double> p, nrm, at, nd;
    bool front;
    hit_record<false, double>(sc, k, o, d, t, p, nrm, front);
    if (!scatter<false, double>(sc, k, d, nrm, front, g, at, nd)) break;
    att[n_att++] = at;
    o = p;
    d = nd;
  }
  for (int q = n_att - 1; q >= 0; q--) col = mk(att[q].x * col.x, att[q].y * col.y, att[q].z * col.z);
  return col;
}

__global__ void replay_kernel(const double4 *__restrict__ geom, const double4 *__restrict__ sh0,
                              const double4 *__restrict__ sh1, ReplayArgs a, const int32_t *__restrict__ ranges,
                              const int32_t *__restrict__ streams, const int64_t *__restrict__ offs,
                              const int64_t *__restrict__ out_offs, double *__restrict__ out,
                              int64_t *__restrict__ used) {
  const int job = blockIdx.x * blockDim.x + threadIdx.x;
  if (job >= a.n_jobs) return;
  const SceneView<double> sc{geom, sh0, sh1, a.n};
  StreamRng g{streams, offs[job], offs[job + 1], false};
  const int start = ranges[2 * job], end = ranges[2 * job + 1];
  double *o = out + out_offs[job];
  for (int index = start; index < end; index++) {  // worker() main.cpp:273-289
    const int j = index / a.W, i = index % a.W;
    V3<double> sum = mk(0.0, 0.0, 0.0);
    for (int s = 0; s < a.spp; s++) {
      const double u = (i + g.uni()) / (a.W - 1);
      const double v = (j + g.uni()) / (a.H - 1);
      V3<double> ro, rd;
      get_ray<false, double>(a.cam, u, v, g, ro, rd);
      const V3<double> c = ray_color_exact(sc, ro, rd, a.max_depth, g);
      sum = mk(sum.x + c.x, sum.y + c.y, sum.z + c.z);
    }
    o[3 * (index - start) + 0] = sum.x;
    o[3 * (index - start) + 1] = sum.y;
    o[3 * (index - start) + 2] = sum.z;
  }
  used[job] = g.overflow ? -1 : g.pos - offs[job];
}

}  // namespace rtmi

// ===========================================================================
// host side
// ===========================================================================
using namespace rtmi;

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return set_error(RT_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int32_t n = 0;
  float4 *geom = nullptr, *sh0 = nullptr, *sh1 = nullptr;
  SpherePair *pairs = nullptr;
  int32_t npairs = 0;
  double4 *geom64 = nullptr, *sh064 = nullptr, *sh164 = nullptr;
  unsigned long long *accum = nullptr;
  size_t accum_cap = 0;  // elements
  float *scratch = nullptr;
  size_t scratch_cap = 0;  // elements
  unsigned long long *segments = nullptr;  // world.hit calls of the last render
  unsigned *counter = nullptr;             // persistent kernel's work-item counter
  int32_t kernel = RT_KERNEL_AUTO;         // RT_KERNEL_* (rtmi.h)
  unsigned long long *pass_accum = nullptr;  // progressive accumulator (fixed point)
  size_t pass_cap = 0;
  int32_t pass_W = 0, pass_rows = 0, pass_spp = 0;
  int32_t resident_blocks = 0;             // blocks of the persistent grid (from the occupancy query)
  int32_t cu_count = 0;                    // compute units of the device
  int32_t res_blocks = 0;                  // resident render_resident blocks for res_lds dynamic LDS bytes
  size_t res_lds = 0;
  // BVH, built by rt_ctx_set_scene
  int32_t accel = RT_ACCEL_GRID;  // the fastest structure (brute force when the scene has none)
  SpherePair *big_pairs = nullptr;
  int32_t *big_idx = nullptr;
  int32_t nbig_pairs = 0, nbig = 0;
  BvhNode *nodes = nullptr;
  int32_t nnodes = 0;
  bool bvh_global = false;  // the BVH is over the LDS budget: walked in global memory
  // RTMI_BVH_GLOBAL=1 (tests): the global-memory walk for any BVH
  bool force_bvh_global = std::getenv("RTMI_BVH_GLOBAL") && std::atoi(std::getenv("RTMI_BVH_GLOBAL")) != 0;
  float4 *bvh_sph = nullptr;
  int32_t *bvh_idx = nullptr;
  int32_t nbvh_sph = 0;
  // uniform grid, built by rt_ctx_set_scene beside the BVH
  float4 *grid_sph = nullptr;  // every sphere by scene index
  uint32_t *grid_cells = nullptr;  // ncells + 1: each cell's first reference
  uint32_t *grid_refs = nullptr;   // 16 x scene index (byte offsets into the LDS sphere array)
  GridDesc grid{};
  int32_t ngrid_sph = 0;
  bool grid_ok = false;
  bool grid_global = false;  // the grid is walked in global memory (grid_gmem: its LDS image)
  char *grid_gmem = nullptr;
  // RTMI_GRID_GLOBAL=1 (tests): the global-memory walk for any grid
  bool force_grid_global = std::getenv("RTMI_GRID_GLOBAL") && std::atoi(std::getenv("RTMI_GRID_GLOBAL")) != 0;
  // cost-ordered dispatch: per-tile world.hit counts of the
  // last render with the same tile layout order the next one's tiles
  int32_t ordering = RT_ORDER_COST;
  // block-level accumulator flush of the automatic grid schedule (same image;
  // RTMI_BLOCK_FLUSH=0 in the environment turns it off, for A/B and tests)
  bool block_flush = !(std::getenv("RTMI_BLOCK_FLUSH") && std::getenv("RTMI_BLOCK_FLUSH")[0] == '0');
  // a block that covers all samples of its tile writes the floats itself
  // (RTMI_BLOCK_OWNS=0 routes it through the accumulator, for A/B and tests)
  bool block_owns = !(std::getenv("RTMI_BLOCK_OWNS") && std::getenv("RTMI_BLOCK_OWNS")[0] == '0');
  // the schedule of the last launch (rt_ctx_last_schedule, for tests)
  int32_t last_sched[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned *cost_prev = nullptr, *cost_cur = nullptr, *cost_sorted = nullptr;
  int32_t *order = nullptr, *iota = nullptr;
  size_t cost_cap = 0;  // tiles
  void *sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  bool cost_valid = false;
  int64_t cost_key[6] = {0, 0, 0, 0, 0, 0};  // W, H, row0, row_step, nvalid, tile_w
  hipStream_t last_stream = nullptr;
  hipEvent_t last_done = nullptr;  // end of the last render's work on last_stream
  int32_t tile_w = 0;  // 0 = automatic per launch (auto_tile_w)
  int32_t chunk = 0;       // phase-1 samples per item (0 = automatic)
  int32_t tail_spp = -1;   // samples in the short-item phase (-1 = automatic)
  int32_t tail_chunk = 0;  // phase-2 samples per item (0 = automatic)
  // cost probe: a render with no cost map of its own tile
  // layout first renders probe_spp samples per pixel into its output strip,
  // counting world.hit per tile, and orders its tiles by those counts.
  // RTMI_ORDER_PROBE: 0 = never probe (order by the previous identical render
  // only), 1 = probe when no map of this layout exists (default), 2 = probe
  // before every render (no state carried between renders)
  int32_t probe_mode = std::getenv("RTMI_ORDER_PROBE") ? std::atoi(std::getenv("RTMI_ORDER_PROBE")) : 1;
  // samples per pixel of the probe (RTMI_PROBE_SPP, for A/B; 0 = automatic)
  int32_t probe_spp = std::getenv("RTMI_PROBE_SPP") ? std::atoi(std::getenv("RTMI_PROBE_SPP")) : 0;
  // path depth limit of the probe (RTMI_PROBE_DEPTH overrides, for A/B and
  // tests; 0 = the default, 8): a tile's cost shows by depth 8 (depth 2 would
  // hide the glass spheres' long paths), and the probe's launch ends sooner
  // without the rare 50-segment paths (one rank's 1/8 strip of config 2,
  // one-shot 2.81 ms with 1 spp to depth 8 against 2.96 with 2 spp to depth
  // 50; the frame 19.57 vs 19.64; profiles/r06/oneshot/)
  int32_t probe_depth = std::getenv("RTMI_PROBE_DEPTH") ? std::atoi(std::getenv("RTMI_PROBE_DEPTH")) : 0;
  bool probing = false;
  // automatic item size of the grid kernel: ~want_items items of item_min..125
  // samples; 0 = the default of the launch mode below (RTMI_WANT_ITEMS /
  // RTMI_ITEM_MIN override, for A/B)
  int64_t want_items = std::getenv("RTMI_WANT_ITEMS") ? std::atoll(std::getenv("RTMI_WANT_ITEMS")) : 0;
  int32_t item_min = std::getenv("RTMI_ITEM_MIN") ? std::atoi(std::getenv("RTMI_ITEM_MIN")) : 0;
  // rt_ctx_set_overlap: this context's launches run beside another context's
  // on the same device, so a launch's dispatch tail is filled by the other's
  // blocks and fewer, longer items pay less per-item overhead
  bool overlap = false;
};

namespace rtmi {
hipStream_t ctx_stream(rt_ctx *ctx) { return ctx->stream; }
}  // namespace rtmi

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

Cam<float> cam_f(const rt_camera *c) {
  auto v = [](const double *p) { return mk(float(p[0]), float(p[1]), float(p[2])); };
  return Cam<float>{v(c->origin), v(c->lower_left_corner), v(c->horizontal), v(c->vertical), v(c->u), v(c->v),
                    float(c->lens_radius)};
}
Cam<double> cam_d(const rt_camera *c) {
  auto v = [](const double *p) { return mk(p[0], p[1], p[2]); };
  return Cam<double>{v(c->origin), v(c->lower_left_corner), v(c->horizontal), v(c->vertical), v(c->u), v(c->v),
                     c->lens_radius};
}

template <class T> int dev_alloc(T **p, size_t count) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), count * sizeof(T));
  if (e != hipSuccess) return set_error(RT_ENOMEM, "hipMalloc(%zu B): %s", count * sizeof(T), hipGetErrorString(e));
  return RT_OK;
}

int check_render_args(const rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp, int32_t max_depth) {
  if (!ctx || !cam) return set_error(RT_EINVAL, "null context or camera");
  if (W < 2 || H < 2) return set_error(RT_EINVAL, "image must be at least 2x2 (u,v divide by W-1, H-1)");
  if (spp < 1 || spp >= (1 << 24)) return set_error(RT_EINVAL, "spp must be in [1, 2^24)");
  if (max_depth < 0 || max_depth >= (1 << 24)) return set_error(RT_EINVAL, "max_depth must be in [0, 2^24)");
  if (int64_t(W) * int64_t(H) >= (int64_t(1) << 40)) return set_error(RT_EINVAL, "image too large");
  if (ctx->n <= 0) return set_error(RT_EINVAL, "no scene uploaded (rt_ctx_set_scene)");
  return RT_OK;
}

}  // namespace

RTMI_EXPORT int rt_device_count(int32_t *n) {
  if (!n) return set_error(RT_EINVAL, "null");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return set_error(RT_ENODEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *n = c;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_create(int32_t device, rt_ctx **out) {
  if (!out) return set_error(RT_EINVAL, "null out");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return set_error(RT_ENODEVICE, "no HIP device visible");
  if (device < 0 || device >= count) return set_error(RT_ENODEVICE, "device %d out of range [0,%d)", device, count);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(RT_ENODEVICE, "device %d is %s; librtmi is built for gfx950 only", device, prop.gcnArchName);
  DeviceGuard guard(device);
  auto ctx = std::make_unique<rt_ctx>();
  ctx->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming));
  if (int rc = dev_alloc(&ctx->segments, 8)) return rc;
  HIP_TRY(hipMemset(ctx->segments, 0, 8 * sizeof(unsigned long long)));
  if (int rc = dev_alloc(&ctx->counter, 1)) return rc;
  {
    // resident blocks per CU for the persistent grid; over-subscription is
    // harmless (extra waves start later and find the counter exhausted)
    int per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)render_persistent<8, true>,
                                                         64 * kWavesPerBlock, 0));
    ctx->resident_blocks = std::max(1, per_cu) * prop.multiProcessorCount;
    ctx->cu_count = prop.multiProcessorCount;
  }
  *out = ctx.release();
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_destroy(rt_ctx *ctx) {
  if (!ctx) return RT_OK;
  DeviceGuard guard(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (void *p : {(void *)ctx->geom, (void *)ctx->sh0, (void *)ctx->sh1, (void *)ctx->geom64, (void *)ctx->sh064,
                  (void *)ctx->sh164, (void *)ctx->accum, (void *)ctx->scratch, (void *)ctx->segments, (void *)ctx->pairs, (void *)ctx->counter, (void *)ctx->pass_accum,
                  (void *)ctx->big_pairs, (void *)ctx->big_idx, (void *)ctx->nodes, (void *)ctx->bvh_sph, (void *)ctx->bvh_idx,
                  (void *)ctx->cost_prev, (void *)ctx->cost_cur, (void *)ctx->cost_sorted, (void *)ctx->order,
                  (void *)ctx->iota, ctx->sort_tmp, (void *)ctx->grid_sph, (void *)ctx->grid_cells, (void *)ctx->grid_refs,
                  (void *)ctx->grid_gmem})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(ctx->stream);
  if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
  delete ctx;
  return RT_OK;
}

namespace {
constexpr size_t kBvhLdsMax = 64 * 1024;  // BVH bytes staged per block

// BVH over the small spheres: binary, SAH split (full sweep of the sorted
// centroids on each axis: the split minimising area(L)*|L| + area(R)*|R|),
// leaves of <= kLeafMax spheres, nodes in DFS order with skip links.  Boxes
// are the spheres' double-precision bounds, each grown by its own margin (1e-3
// of the sphere's coordinate scale, ~100x the float error of its hit test,
// plus 1e-6 of the scene's) and rounded outward to half precision, so every
// sphere the float test can report lies strictly inside its leaf's box.
uint16_t half_bits(_Float16 h) { return __builtin_bit_cast(uint16_t, h); }
// largest half <= v (-inf below the half range)
uint16_t half_down(double v) {
  _Float16 h = _Float16(v);
  while (double(h) > v) {
    uint16_t b = half_bits(h);
    if (b == 0x0000) b = 0x8001;          // +0 -> -min denormal
    else if (b & 0x8000) b = uint16_t(b + 1);  // negative: away from zero
    else b = uint16_t(b - 1);             // positive: toward zero
    h = __builtin_bit_cast(_Float16, b);
  }
  return half_bits(h);
}
uint16_t half_up(double v) { return uint16_t(half_down(-v) ^ 0x8000); }

struct BvhBuilder {
  const double *cr;
  const std::vector<float4> &g;
  double margin_scene;  // 1e-6 of the whole scene's scale (rays from far away)
  std::vector<BvhNode> nodes;
  std::vector<float4> sph;
  std::vector<int32_t> idx;

  struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void add(const double *c, double rr) {
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], c[a] - rr);
        hi[a] = std::max(hi[a], c[a] + rr);
      }
    }
    double area() const {
      const double e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
      return e0 * e1 + e1 * e2 + e0 * e2;
    }
  };
  // sphere k's box margin: 1e-3 of its own coordinate scale (~100x the float
  // error of its hit test) + margin_scene
  double margin(int32_t k) const {
    const double *c = cr + 4 * k;
    const double own = std::max(std::max(std::fabs(c[0]), std::fabs(c[1])), std::fabs(c[2])) + std::fabs(c[3]);
    return 1e-3 * (1.0 + own) + margin_scene;
  }
  Box bounds(const int32_t *ids, int cnt) const {
    Box b;
    for (int i = 0; i < cnt; ++i) b.add(cr + 4 * ids[i], std::fabs(cr[4 * ids[i] + 3]) + margin(ids[i]));
    return b;
  }
  void sort_axis(int32_t *ids, int cnt, int ax) const {
    std::sort(ids, ids + cnt, [&](int32_t x, int32_t y) {
      const double cx = cr[4 * x + ax], cy = cr[4 * y + ax];
      return cx < cy || (cx == cy && x < y);
    });
  }
  void build(int32_t *ids, int cnt) {
    const int me = int(nodes.size());
    nodes.push_back(BvhNode{});
    const Box bb = bounds(ids, cnt);
    BvhNode nd{};
    nd.x = uint32_t(half_down(bb.lo[0])) | uint32_t(half_up(bb.hi[0])) << 16;
    nd.y = uint32_t(half_down(bb.lo[1])) | uint32_t(half_up(bb.hi[1])) << 16;
    nd.z = uint32_t(half_down(bb.lo[2])) | uint32_t(half_up(bb.hi[2])) << 16;
    if (cnt <= kLeafMax) {
      nd.link = ~((int32_t(sph.size()) << 4) | cnt);
      for (int i = 0; i < cnt; ++i) {
        sph.push_back(g[ids[i]]);
        idx.push_back(ids[i]);
      }
    } else {
      // SAH sweep: prefix/suffix boxes over the centroid order of each axis
      double best = INFINITY;
      int best_ax = 0, best_mid = cnt / 2;
      std::vector<double> left_cost(cnt);
      for (int ax = 0; ax < 3; ++ax) {
        sort_axis(ids, cnt, ax);
        Box l;
        for (int i = 1; i < cnt; ++i) {
          l.add(cr + 4 * ids[i - 1], std::fabs(cr[4 * ids[i - 1] + 3]) + margin(ids[i - 1]));
          left_cost[i] = l.area() * i;
        }
        Box r;
        for (int i = cnt - 1; i >= 1; --i) {
          r.add(cr + 4 * ids[i], std::fabs(cr[4 * ids[i] + 3]) + margin(ids[i]));
          const double c = left_cost[i] + r.area() * (cnt - i);
          if (c < best) { best = c; best_ax = ax; best_mid = i; }
        }
      }
      sort_axis(ids, cnt, best_ax);
      build(ids, best_mid);
      build(ids + best_mid, cnt - best_mid);
      nd.link = int32_t(nodes.size());
    }
    nodes[me] = nd;
  }
};
}  // namespace

namespace {
// Uniform grid over the small spheres.  The box of their
// margin-grown boxes (the BVH's margins) is cut into cells of about
// RTMI_GRID_CELLS (default 0.3) cells per sphere, as near cubic as the box
// allows (the final scene's thin layer of spheres: 30 x 1 x 30 cells); every
// sphere is listed in every cell its grown box overlaps.  Cell boundaries are
// the float values g0 + c*h the device computes, so host and device agree to
// a rounding error far below the margins.
struct GridBuild {
  GridDesc desc{};
  std::vector<float4> sph;     // every sphere of the scene by scene index
  std::vector<uint32_t> cells;  // ncells + 1: each cell's first reference
  std::vector<uint32_t> refs;   // 16 x scene index
  bool fits_lds = true;         // its LDS image fits the per-block budget (else: walked in global memory)
};
bool build_grid(const BvhBuilder &b, const std::vector<int32_t> &small, int32_t n, int32_t nbig_slots,
                GridBuild &out) {
  if (n > 65535) return false;  // references are 16-bit scene indices
  const char *env = std::getenv("RTMI_GRID_CELLS");
  // 0.3 cells per sphere: config 2 33.3 ms (0.2: 33.3, 0.5: 33.6, 1: 34.5,
  // 2: 35.2, 4: 38.0; round 2) and, on the record slots, 19.30 ms (0.2:
  // 19.38, 0.25: 19.33, 0.4: 19.33; profiles/r04/grid_density.txt)
  const double per_sphere = env && std::atof(env) > 0 ? std::atof(env) : 0.3;
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int32_t k : small) {
    const double *c = b.cr + 4 * k, R = std::fabs(c[3]) + b.margin(k);
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], c[a] - R);
      hi[a] = std::max(hi[a], c[a] + R);
    }
  }
  double e[3], vol = 1;
  for (int a = 0; a < 3; ++a) {
    e[a] = std::max(hi[a] - lo[a], 1e-6 * (1 + std::fabs(lo[a])));
    vol *= e[a];
  }
  const double cell = std::cbrt(vol / (per_sphere * double(small.size())));
  // analysis knob: RTMI_GRID_ASPECT = x-cell / z-cell size ratio (1: cubic)
  const char *asp_env = std::getenv("RTMI_GRID_ASPECT");
  const double asp = asp_env && std::atof(asp_env) > 0 ? std::atof(asp_env) : 1.0;
  const double cell_a[3] = {cell * std::sqrt(asp), cell, cell / std::sqrt(asp)};
  int64_t total = 1;
  for (int a = 0; a < 3; ++a) {
    out.desc.n[a] = int32_t(std::min<double>(128, std::max<double>(1, std::ceil(e[a] / cell_a[a]))));
    total *= out.desc.n[a];
  }
  if (total > 16384) return false;
  for (int a = 0; a < 3; ++a) {
    // origin rounded down, cell size rounded up: the float cells cover the box
    float g0 = float(lo[a]);
    if (double(g0) > lo[a]) g0 = std::nextafter(g0, -INFINITY);
    float h = float(e[a] / out.desc.n[a]);
    while (double(g0) + double(h) * out.desc.n[a] < hi[a]) h = std::nextafter(h, INFINITY);
    out.desc.g0[a] = g0;
    out.desc.h[a] = h;
    out.desc.inv_h[a] = 1.0f / h;
    out.desc.g1[a] = std::fmaf(float(out.desc.n[a]), h, g0);
  }
  out.desc.ncells = int32_t(total);
  std::vector<std::vector<uint16_t>> lists(static_cast<size_t>(total));
  for (int32_t k : small) {  // ascending scene index
    const double *c = b.cr + 4 * k, R = std::fabs(c[3]) + b.margin(k);
    int c0[3], c1[3];
    for (int a = 0; a < 3; ++a) {
      // cell c spans [g0 + c*h, g0 + (c+1)*h]: every cell the grown box touches
      const double g0 = out.desc.g0[a], h = out.desc.h[a];
      c0[a] = std::max(0, std::min(out.desc.n[a] - 1, int(std::floor((c[a] - R - g0) / h))));
      c1[a] = std::max(0, std::min(out.desc.n[a] - 1, int(std::floor((c[a] + R - g0) / h))));
    }
    for (int z = c0[2]; z <= c1[2]; ++z)
      for (int y = c0[1]; y <= c1[1]; ++y)
        for (int x = c0[0]; x <= c1[0]; ++x)
          lists[size_t(x + out.desc.n[0] * (y + out.desc.n[1] * z))].push_back(uint16_t(k));
  }
  // the LDS sphere array: the scene's spheres at their scene indices
  out.sph.assign(b.g.begin(), b.g.begin() + n);
  out.cells.resize(size_t(total) + 1);
  for (int64_t cidx = 0; cidx < total; ++cidx) {
    out.cells[size_t(cidx)] = uint32_t(out.refs.size());
    for (uint16_t k : lists[size_t(cidx)]) out.refs.push_back(uint32_t(k) * 16u);
  }
  out.cells[size_t(total)] = uint32_t(out.refs.size());
  out.desc.nrefs = int32_t(out.refs.size());
  out.desc.cells_off = 16u * uint32_t(nbig_slots + out.desc.nrefs);  // grid_lds_bytes' layout
  out.desc.idx_off = out.desc.cells_off + 4u * uint32_t(out.desc.ncells + 1);
  // The grid is staged in LDS only while a 4-wave block (its grid copy, one
  // accumulator set, the static LDS) still leaves 8 blocks per CU; a larger
  // one is walked in global memory (Accel::grid_gmem).  Measured
  // (tools/large_scene_bench.py, profiles/r05/large/): the final scene's
  // 17.6 KB grid 1.05 ms in LDS vs 1.13 in global memory (config 2: 19.2 vs
  // 20.2 ms); 1 604 spheres (a 58 KB grid, 2 blocks per CU) 2.71 vs 1.13 ms.
  // RTMI_GRID_LDS_MAX overrides the byte limit (A/B).
  const char *lim_env = std::getenv("RTMI_GRID_LDS_MAX");
  const size_t lds_max = lim_env && std::atoll(lim_env) > 0 ? size_t(std::atoll(lim_env)) : 160 * 1024 / 8 - 3 * 64 * 8 - 256;
  out.fits_lds = grid_lds_bytes(nbig_slots, out.desc.ncells, out.desc.nrefs) <= lds_max;
  return true;
}
}  // namespace

RTMI_EXPORT int rt_ctx_set_ordering(rt_ctx *ctx, int32_t ordering) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (ordering != RT_ORDER_NONE && ordering != RT_ORDER_COST) return set_error(RT_EINVAL, "unknown ordering %d", ordering);
  ctx->ordering = ordering;
  ctx->cost_valid = false;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_set_accel(rt_ctx *ctx, int32_t accel) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (accel != RT_ACCEL_NONE && accel != RT_ACCEL_BVH && accel != RT_ACCEL_GRID)
    return set_error(RT_EINVAL, "unknown accel %d", accel);
  ctx->accel = accel;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_accel_info(rt_ctx *ctx, int32_t *n_big, int32_t *n_nodes) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (n_big) *n_big = ctx->nbig;
  if (n_nodes) *n_nodes = ctx->nnodes;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_set_scene(rt_ctx *ctx, const rt_scene *scene) {
  if (!ctx || !scene || scene->n <= 0 || !scene->center_radius || !scene->mat_kind || !scene->mat_params)
    return set_error(RT_EINVAL, "rt_ctx_set_scene: bad argument");
  const int n = scene->n;
  std::vector<float4> g(n + kGeomPad, make_float4(0.f, 0.f, 0.f, 0.f)), s0(n), s1(n);
  std::vector<double4> g64(n), s064(n), s164(n);
  for (int k = 0; k < n; k++) {
    const double *c = scene->center_radius + 4 * k;
    const double *m = scene->mat_params + 4 * k;
    const int kind = scene->mat_kind[k];
    if (kind < RT_MAT_LAMBERTIAN || kind > RT_MAT_DIELECTRIC)
      return set_error(RT_EUNSUPPORTED, "object %d: unsupported material kind %d", k, kind);
    const double fuzz = m[3] < 1 ? m[3] : 1;  // metal ctor material.h:39
    const float r = float(c[3]), ir = float(m[3]);
    // S = |c|^2 - r^2 of the float-rounded sphere, in double then rounded
    // (the oracle computes the identical expression)
    const float cx = float(c[0]), cy = float(c[1]), cz = float(c[2]);
    const float S = float(double(cx) * cx + double(cy) * cy + double(cz) * cz - double(r) * r);
    g[k] = make_float4(cx, cy, cz, S);
    s0[k] = make_float4(1.0f / r, float(m[0]), float(m[1]), float(m[2]));
    s1[k] = make_float4(float(kind), float(fuzz), ir, 1.0f / ir);
    if (kind == RT_MAT_DIELECTRIC) {
      // Schlick's r0 for both faces (material.h:91-96), in the float
      // arithmetic the kernels would repeat per scatter: front (ratio 1/ir)
      // in shade1.y, back (ratio ir) in shade0.y — fields a dielectric does
      // not otherwise read (no albedo, no fuzz)
      auto r0_of = [](float x) {
        const float q = (1.0f - x) / (1.0f + x);
        return q * q;
      };
      s1[k].y = r0_of(1.0f / ir);
      s0[k].y = r0_of(ir);
    }
    g64[k] = make_double4(c[0], c[1], c[2], c[3] * c[3]);
    s064[k] = make_double4(1 / c[3], m[0], m[1], m[2]);
    s164[k] = make_double4(double(kind), fuzz, m[3], 1.0 / m[3]);
  }
  // sphere pairs for the packed loop: n padded to a multiple of 2*kPairGroup
  // with never-hit dummies, plus kPairGroup pairs of prefetch padding
  const int n_pad = (n + 2 * kPairGroup - 1) / (2 * kPairGroup) * (2 * kPairGroup);
  const int npairs = n_pad / 2;
  std::vector<SpherePair> pr(npairs + kPairGroup);
  for (auto &p : pr) {
    p.cx = f2v{0.f, 0.f}; p.cy = f2v{0.f, 0.f}; p.cz = f2v{0.f, 0.f}; p.S = f2v{kDummyS, kDummyS};
  }
  for (int k = 0; k < n; k++) {
    SpherePair &p = pr[k / 2];
    const int h = k & 1;
    p.cx[h] = g[k].x; p.cy[h] = g[k].y; p.cz[h] = g[k].z; p.S[h] = g[k].w;
  }
  DeviceGuard guard(ctx->device);
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  int rc;
  if ((rc = dev_alloc(&ctx->geom, n + kGeomPad)) || (rc = dev_alloc(&ctx->sh0, n)) || (rc = dev_alloc(&ctx->sh1, n)) ||
      (rc = dev_alloc(&ctx->geom64, n)) || (rc = dev_alloc(&ctx->sh064, n)) || (rc = dev_alloc(&ctx->sh164, n)) ||
      (rc = dev_alloc(&ctx->pairs, pr.size())))
    return rc;
  HIP_TRY(hipMemcpy(ctx->pairs, pr.data(), pr.size() * sizeof(SpherePair), hipMemcpyHostToDevice));
  ctx->npairs = npairs;
  HIP_TRY(hipMemcpy(ctx->geom, g.data(), (n + kGeomPad) * sizeof(float4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->sh0, s0.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->sh1, s1.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->geom64, g64.data(), n * sizeof(double4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->sh064, s064.data(), n * sizeof(double4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->sh164, s164.data(), n * sizeof(double4), hipMemcpyHostToDevice));
  // BVH: spheres much larger than the typical one (the ground) stay brute force
  {
    std::vector<double> rad(n);
    for (int k = 0; k < n; k++) rad[k] = std::fabs(scene->center_radius[4 * k + 3]);
    std::vector<double> sorted_r = rad;
    std::nth_element(sorted_r.begin(), sorted_r.begin() + n / 2, sorted_r.end());
    const double med = sorted_r[n / 2];
    std::vector<int32_t> big, small;
    double scale = 0;  // the whole scene's, big spheres included
    for (int k = 0; k < n; k++) {
      (rad[k] > RTMI_BIG_FACTOR * med ? big : small).push_back(k);
      for (int a = 0; a < 3; ++a) scale = std::max(scale, std::fabs(scene->center_radius[4 * k + a]) + rad[k]);
    }
    BvhBuilder b{scene->center_radius, g, 1e-6 * scale, {}, {}, {}};
    if (!small.empty()) b.build(small.data(), int(small.size()));
    const int nb_pad = big.empty() ? 0 : (int(big.size()) + 2 * kBigGroup - 1) / (2 * kBigGroup) * (2 * kBigGroup);
    std::vector<SpherePair> bp(nb_pad / 2 + kPairGroup);
    std::vector<int32_t> bidx(size_t(nb_pad) + 2 * kPairGroup, -1);
    for (auto &p : bp) {
      p.cx = f2v{0.f, 0.f}; p.cy = f2v{0.f, 0.f}; p.cz = f2v{0.f, 0.f}; p.S = f2v{kDummyS, kDummyS};
    }
    for (size_t s = 0; s < big.size(); s++) {  // ascending scene index
      SpherePair &p = bp[s / 2];
      const int h = int(s & 1), k = big[s];
      p.cx[h] = g[k].x; p.cy[h] = g[k].y; p.cz[h] = g[k].z; p.S[h] = g[k].w;
      bidx[s] = k;
    }
    if ((rc = dev_alloc(&ctx->big_pairs, bp.size())) || (rc = dev_alloc(&ctx->big_idx, bidx.size())) ||
        (rc = dev_alloc(&ctx->nodes, std::max<size_t>(b.nodes.size(), 1))) ||
        (rc = dev_alloc(&ctx->bvh_sph, std::max<size_t>(b.sph.size(), 1))) ||
        (rc = dev_alloc(&ctx->bvh_idx, std::max<size_t>(b.idx.size(), 1))))
      return rc;
    HIP_TRY(hipMemcpy(ctx->big_pairs, bp.data(), bp.size() * sizeof(SpherePair), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ctx->big_idx, bidx.data(), bidx.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!b.nodes.empty()) {
      HIP_TRY(hipMemcpy(ctx->nodes, b.nodes.data(), b.nodes.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(ctx->bvh_sph, b.sph.data(), b.sph.size() * sizeof(float4), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(ctx->bvh_idx, b.idx.data(), b.idx.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    ctx->nbig = int32_t(big.size());
    ctx->nbig_pairs = nb_pad / 2;
    ctx->nbvh_sph = int32_t(b.sph.size());
    // the BVH is staged in LDS while a block (BVH, one accumulator set, the
    // static LDS) still leaves 8 blocks per CU and its 16-bit scene indices
    // suffice; a larger one is walked in global memory (L2).  Measured
    // (profiles/r05/large/threshold_ab.txt): 488 spheres 1.90 ms in LDS vs
    // 2.06 global, 904 spheres 2.33 vs 2.34, 1 604 spheres 3.74 vs 2.42.
    // RTMI_BVH_LDS_MAX overrides the byte limit (A/B).
    const size_t lds = bvh_lds_bytes(int32_t(b.nodes.size()), int32_t(b.sph.size()));
    const char *lim_env = std::getenv("RTMI_BVH_LDS_MAX");
    const size_t lds_max = lim_env && std::atoll(lim_env) > 0 ? std::min<size_t>(kBvhLdsMax, size_t(std::atoll(lim_env)))
                                                             : 160 * 1024 / 8 - 3 * 64 * 8 - 256;
    ctx->nnodes = int32_t(b.nodes.size());
    ctx->bvh_global = ctx->force_bvh_global || !(lds <= lds_max && n <= 65535);
    // uniform grid over the same small spheres
    ctx->grid_ok = false;
    GridBuild gb;
    if (!small.empty() && build_grid(b, small, n, nb_pad, gb)) {
      if ((rc = dev_alloc(&ctx->grid_sph, gb.sph.size())) || (rc = dev_alloc(&ctx->grid_cells, gb.cells.size())) ||
          (rc = dev_alloc(&ctx->grid_refs, std::max<size_t>(gb.refs.size(), 1))))
        return rc;
      HIP_TRY(hipMemcpy(ctx->grid_sph, gb.sph.data(), gb.sph.size() * sizeof(float4), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(ctx->grid_cells, gb.cells.data(), gb.cells.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      if (!gb.refs.empty())
        HIP_TRY(hipMemcpy(ctx->grid_refs, gb.refs.data(), gb.refs.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      ctx->grid = gb.desc;
      ctx->grid.cells = ctx->grid_cells;
      ctx->grid.refs = ctx->grid_refs;
      ctx->ngrid_sph = int32_t(gb.sph.size());
      ctx->grid_global = ctx->force_grid_global || !gb.fits_lds;
      if (ctx->grid_global) {
        // the image stage_grid builds in LDS, offsets from 0: the slots (big
        // spheres, then every cell's references as copies of their spheres'
        // records), the cell starts, the slots' scene indices
        const int32_t nbs = nb_pad, nrec = nbs + gb.desc.nrefs;
        std::vector<char> img(grid_lds_bytes(nbs, gb.desc.ncells, gb.desc.nrefs), 0);
        float4 *rec = reinterpret_cast<float4 *>(img.data());
        uint32_t *cst = reinterpret_cast<uint32_t *>(img.data() + gb.desc.cells_off);
        uint16_t *ix = reinterpret_cast<uint16_t *>(img.data() + gb.desc.idx_off);
        for (int32_t i = 0; i < nrec; ++i) {
          const int32_t k = i < nbs ? bidx[size_t(i)] : int32_t(gb.refs[size_t(i - nbs)] >> 4);  // dummies: -1
          rec[i] = k < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : gb.sph[size_t(k)];
          ix[i] = uint16_t(k < 0 ? 0 : k);
        }
        for (int32_t i = 0; i <= gb.desc.ncells; ++i) cst[i] = 16u * (uint32_t(nbs) + gb.cells[size_t(i)]);
        if ((rc = dev_alloc(&ctx->grid_gmem, img.size()))) return rc;
        HIP_TRY(hipMemcpy(ctx->grid_gmem, img.data(), img.size(), hipMemcpyHostToDevice));
      }
      ctx->grid_ok = true;
    }
  }
  ctx->n = n;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_grid_info(rt_ctx *ctx, int32_t *dims3, int32_t *n_refs, int32_t *lds_bytes) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (!ctx->grid_ok) return set_error(RT_EUNSUPPORTED, "no grid for this scene");
  if (dims3) for (int a = 0; a < 3; ++a) dims3[a] = ctx->grid.n[a];
  if (n_refs) *n_refs = ctx->grid.nrefs;
  if (lds_bytes) *lds_bytes = int32_t(grid_lds_bytes(2 * ctx->nbig_pairs, ctx->grid.ncells, ctx->grid.nrefs));
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_set_schedule(rt_ctx *ctx, int32_t chunk, int32_t tail_spp, int32_t tail_chunk) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (chunk < 0 || tail_chunk < 0) return set_error(RT_EINVAL, "chunk sizes must be >= 0");
  ctx->chunk = chunk;
  ctx->tail_spp = tail_spp;
  ctx->tail_chunk = tail_chunk;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_set_overlap(rt_ctx *ctx, int32_t overlapped) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (overlapped != 0 && overlapped != 1) return set_error(RT_EINVAL, "overlapped must be 0 or 1");
  ctx->overlap = overlapped != 0;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_set_kernel(rt_ctx *ctx, int32_t kind) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (kind != RT_KERNEL_GRID && kind != RT_KERNEL_PERSISTENT && kind != RT_KERNEL_AUTO && kind != RT_KERNEL_QUEUE &&
      kind != RT_KERNEL_RESIDENT)
    return set_error(RT_EINVAL, "unknown kernel kind");
  ctx->kernel = kind;
  return RT_OK;
}

// Automatic tile shape: 8x8 unless 16x4 leaves fewer idle lanes in partial
// tiles.  A 100-row strip (1/8 of config 2's rows) fills 25 rows of 16x4 tiles
// but 12.5 of 8x8: 7.04 vs 7.16 ms, while the whole frame runs 50.6 ms with 8x8
// and 50.9 with 16x4 (profiles/r01/session6/tile_ab.txt).
static int auto_tile_w(int32_t W, int32_t rows) {
  auto idle = [&](int64_t tw) {
    const int64_t th = 64 / tw;
    return ((W + tw - 1) / tw) * tw * ((rows + th - 1) / th) * th - int64_t(W) * rows;
  };
  return idle(16) < idle(8) ? 16 : 8;
}

RTMI_EXPORT int rt_ctx_set_tuning(rt_ctx *ctx, int32_t tile_w, int32_t chunk) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (tile_w != 0 && tile_w != 8 && tile_w != 16 && tile_w != 32 && tile_w != 64)
    return set_error(RT_EINVAL, "tile_w must be 0 (automatic), 8, 16, 32 or 64");
  if (chunk < 0) return set_error(RT_EINVAL, "chunk must be >= 0");
  ctx->tile_w = tile_w;
  ctx->chunk = chunk;
  return RT_OK;
}

namespace {

size_t accel_lds_bytes(const Accel &acc, int kind) {
  if (kind == 1) return acc.bvh_global ? 0 : bvh_lds_bytes(acc.nnodes, acc.nsph);
  if (kind >= 4) return 0;  // (the grid in global memory)
  if (kind >= 2) return grid_lds_bytes(2 * acc.nbig_pairs, acc.grid.ncells, acc.grid.nrefs);
  return 0;
}

// The Accel view of the context's structure of `kind` (1 BVH, 2 grid, 3 the
// grid walked as one y layer).
Accel accel_of(const rt_ctx *ctx, int kind) {
  Accel a{ctx->big_pairs, ctx->big_idx, ctx->nbig_pairs, 0, nullptr, nullptr, nullptr, 0, GridDesc{}};
  if (kind == 1) {
    a.nnodes = ctx->nnodes;
    a.nodes = ctx->nodes;
    a.sph = ctx->bvh_sph;
    a.sph_idx = ctx->bvh_idx;
    a.nsph = ctx->nbvh_sph;
    a.bvh_global = ctx->bvh_global;
  } else if (kind >= 2) {
    a.sph = ctx->grid_sph;
    a.nsph = ctx->ngrid_sph;
    a.grid = ctx->grid;
    a.grid_gmem = ctx->grid_global ? ctx->grid_gmem : nullptr;
  }
  return a;
}

template <int TW>
void launch_persistent(bool chunked, dim3 grid, hipStream_t st, const rt_ctx *ctx, const RenderArgs &a,
                       unsigned long long *accum, float *out) {
  if (chunked)
    hipLaunchKernelGGL((render_persistent<TW, true>), grid, dim3(64 * kWavesPerBlock), 0, st, ctx->geom, ctx->sh0,
                       ctx->sh1, ctx->pairs, a, accum, out, ctx->segments, ctx->counter);
  else
    hipLaunchKernelGGL((render_persistent<TW, false>), grid, dim3(64 * kWavesPerBlock), 0, st, ctx->geom, ctx->sh0,
                       ctx->sh1, ctx->pairs, a, accum, out, ctx->segments, ctx->counter);
}

template <int TW, int ACC>
void launch_tw(bool chunked, dim3 grid, hipStream_t st, const rt_ctx *ctx, const RenderArgs &a,
               unsigned long long *accum, float *out) {
  // dynamic LDS: the structure, then the accumulators (render_kernel: one
  // set per block with block_flush, else one per wave)
  RenderArgs b = a;
  b.acc_off = int32_t((accel_lds_bytes(a.acc, ACC) + 15) / 16 * 16);
  const size_t lds = size_t(b.acc_off) + size_t(chunked && a.block_flush ? 1 : GridShape<ACC != 0>::waves) * 3 * 64 * 8;
  if (chunked)
    hipLaunchKernelGGL((render_kernel<TW, true, ACC>), grid, dim3(64 * GridShape<ACC != 0>::waves), lds, st, ctx->geom,
                       ctx->sh0, ctx->sh1, ctx->pairs, b, accum, out, ctx->segments);
  else
    hipLaunchKernelGGL((render_kernel<TW, false, ACC>), grid, dim3(64 * GridShape<ACC != 0>::waves), lds, st, ctx->geom,
                       ctx->sh0, ctx->sh1, ctx->pairs, b, accum, out, ctx->segments);
}

#if RTMI_EXPERIMENTAL
// resident blocks of render_resident with dyn bytes of dynamic LDS
int res_resident_blocks(rt_ctx *ctx, size_t dyn) {
  if (ctx->res_blocks <= 0 || ctx->res_lds != dyn) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)render_resident<8, 3>, 64 * kResWaves,
                                                     dyn) != hipSuccess)
      per_cu = 0;
    ctx->res_blocks = std::max(1, per_cu) * std::max(1, ctx->cu_count);
    ctx->res_lds = dyn;
  }
  return ctx->res_blocks;
}

// dynamic LDS of render_resident: the structure, then one sum set per wave
size_t res_lds_bytes(const Accel &acc, int kind, int32_t *acc_off) {
  *acc_off = int32_t((accel_lds_bytes(acc, kind) + 15) / 16 * 16);
  return size_t(*acc_off) + size_t(kResWaves) * 3 * 64 * 8;
}

template <int TW>
void launch_resident(int acc, dim3 grid, size_t lds, hipStream_t st, const rt_ctx *ctx, const RenderArgs &a,
                     unsigned long long *accum, float *out) {
#define RTMI_GO(K)                                                                                            \
  hipLaunchKernelGGL((render_resident<TW, K>), grid, dim3(64 * kResWaves), lds, st, ctx->geom, ctx->sh0, ctx->sh1, a, \
                     accum, out, ctx->segments, ctx->counter)
  switch (acc) {
    case 1: RTMI_GO(1); break;
    case 2: RTMI_GO(2); break;
    case 3: RTMI_GO(3); break;
    case 4: RTMI_GO(4); break;
    default: RTMI_GO(5); break;
  }
#undef RTMI_GO
}

#endif  // RTMI_EXPERIMENTAL

template <int TW>
void launch_shape(bool persistent, int acc, bool chunked, dim3 grid, hipStream_t st, const rt_ctx *ctx,
                  const RenderArgs &a, unsigned long long *accum, float *out) {
  if (persistent) {  // brute force only
    launch_persistent<TW>(chunked, grid, st, ctx, a, accum, out);
  } else {
    if (acc == 1) launch_tw<TW, 1>(chunked, grid, st, ctx, a, accum, out);
    else if (acc == 2) launch_tw<TW, 2>(chunked, grid, st, ctx, a, accum, out);
    else if (acc == 3) launch_tw<TW, 3>(chunked, grid, st, ctx, a, accum, out);
    else if (acc == 4) launch_tw<TW, 4>(chunked, grid, st, ctx, a, accum, out);
    else if (acc == 5) launch_tw<TW, 5>(chunked, grid, st, ctx, a, accum, out);
    else launch_tw<TW, 0>(chunked, grid, st, ctx, a, accum, out);
  }
}

// The render of one row set into a device strip; all work on `st`.
// With pass_accum set (a progressive pass), samples s_base + [0, spp) are
// added to that fixed-point accumulator ([nrows][W][3]) and nothing is
// written to `strip`.
int render_rows_impl(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp, int32_t max_depth,
                     uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows, float *strip, hipStream_t st,
                     int32_t s_base = 0, unsigned long long *pass_accum = nullptr) {
  // The context's buffers (accumulator, counters, cost maps) are reused by
  // every render: a render on another stream first waits for the last one.
  if (ctx->last_stream && ctx->last_stream != st) HIP_TRY(hipStreamWaitEvent(st, ctx->last_done, 0));
  ctx->last_stream = st;
  struct MarkDone {  // record the end of this render's work, whatever path returns
    rt_ctx *c;
    hipStream_t s;
    ~MarkDone() { (void)hipEventRecord(c->last_done, s); }
  } mark_done{ctx, st};
  HIP_TRY(hipMemsetAsync(ctx->segments, 0, 8 * sizeof(unsigned long long), st));
  if (nrows == 0) return RT_OK;
  // valid rows: row0 + r*row_step < H
  int32_t nvalid = 0;
  if (row0 < H) nvalid = std::min<int64_t>(nrows, (int64_t(H) - row0 + row_step - 1) / row_step);
  if (nvalid < nrows && !pass_accum)
    HIP_TRY(hipMemsetAsync(strip + size_t(nvalid) * W * 3, 0, size_t(nrows - nvalid) * W * 3 * sizeof(float), st));
  if (nvalid == 0 || (pass_accum && spp == 0)) return RT_OK;
  if (max_depth == 0) {  // ray_color returns black before any hit test (main.cpp:58-60)
    if (!pass_accum) HIP_TRY(hipMemsetAsync(strip, 0, size_t(nvalid) * W * 3 * sizeof(float), st));
    return RT_OK;
  }
  const int TW = ctx->tile_w ? ctx->tile_w : auto_tile_w(W, nvalid), TH = 64 / TW;
  const int tiles_x = (W + TW - 1) / TW;
  const int tiles_y = (nvalid + TH - 1) / TH;
  const int64_t tiles = int64_t(tiles_x) * tiles_y;
  // Work items: phase 1 covers the first spp1 samples in
  // long items (chunk1: few per-item ramp-down tails and accumulator flushes),
  // phase 2 the rest in short items (chunk2) that run last, so the grid's
  // dispatch tail is one short item.
  // Automatic: ~150 k items (about 24 per resident wave slot on 256 CUs),
  // items of 16..64 samples; measured on config 2: chunk 50 -> 128.4 ms,
  // 100 -> 133, 167 -> 143, 500 -> 193, 25 -> 133, 10 -> 149.
  // Kernel shape (automatic): the resident persistent grid wins on strips
  // (measured, config 2 rows of 1 rank: 1/2 of the image 65.5 vs 67.3 ms,
  // 1/4 33.4 vs 36.5, 1/8 17.9 vs 19.3); one wave per item on a whole frame
  // (128.2 vs 130.4 ms).  Both give the same image.
  const int64_t tile_samples = tiles * int64_t(spp);
  // accelerated closest hit (1 BVH, 2 grid; 0 brute force) when the scene
  // has one; both stage their structure in LDS and use the same block shape
  // (3: the grid has one cell layer in y and the grid kernel walks it with
  // the y stepping dropped, hit_world_grid<.., true>: the same cells, 3% faster
  // on config 2)
  // (a grid that does not fit, e.g. thousands of spheres, leaves the BVH)
  const int acc_kind = ctx->accel == RT_ACCEL_GRID && ctx->grid_ok
                           ? (ctx->grid.n[1] == 1 ? 3 : 2) + (ctx->grid_global ? 2 : 0)
                           : (ctx->accel != RT_ACCEL_NONE && ctx->nnodes > 0 ? 1 : 0);
  const bool bvh = acc_kind != 0;
  // the resident grid kernel: accelerated scenes, when
  // selected, in the experimental build only (measured slower than the grid
  // kernel; the product runs the automatic choice, as for RT_KERNEL_QUEUE,
  // whose kernel was retired in round 6: §4.6)
  const bool resident = RTMI_EXPERIMENTAL && bvh && ctx->kernel == RT_KERNEL_RESIDENT && TW <= 16;
  // the persistent kernel runs brute-force scenes only (see the note above stage_camera)
  const bool persistent = !bvh && (ctx->kernel == RT_KERNEL_PERSISTENT ||
                                   (ctx->kernel == RT_KERNEL_AUTO && tile_samples < 6000000));
  int32_t chunk1 = ctx->chunk, chunk2 = ctx->tail_chunk, tail = ctx->tail_spp;
  if (chunk1 <= 0 && persistent) {
    // ~28 items per resident wave (1/8 strip: chunk 8 -> 17.5 ms, 16 -> 17.9, 32 -> 19.7)
    const int64_t waves = int64_t(ctx->resident_blocks) * kWavesPerBlock;
    chunk1 = int32_t(std::min<int64_t>(64, std::max<int64_t>(4, tile_samples / (28 * waves))));
  } else if (chunk1 <= 0) {
    // ~60 k items of 24..125 samples (BVH, cost order, block flush; the
    // rounding below keeps a multiple of 4 items per tile): config 2 runs
    // 52.5 ms with chunk 21, 51.1 with 42, 50.8 with 63, 50.7 with 125; one
    // rank's 1/8 strip 8.06 ms with 7, 7.37 with 14, 7.18 with 21, 7.27 with
    // 32 (profiles/r01/session6/chunk_ab.txt): long items pay the per-item
    // ramp-down less often, short ones shorten a small grid's dispatch tail
    // With overlapping launches (rt_ctx_set_overlap) ~15 k items of >= 63
    // samples: one rank's strip of config 2 at 1/2, 1/4, 1/8 of the rows
    // 9.54 / 4.89-4.92 / 2.53 ms against 9.87 / 5.14 / 2.64 with the
    // single-launch default (profiles/r05/pipeline/ab_items.txt)
    const int64_t want_items = ctx->want_items > 0 ? ctx->want_items : (ctx->overlap ? 15000 : 60000);
    const int64_t item_min = ctx->item_min > 0 ? ctx->item_min : (ctx->overlap ? 63 : 24);
    chunk1 = int32_t(std::min<int64_t>(125, std::max<int64_t>(item_min, tile_samples / want_items)));
  }
  if (chunk2 <= 0) chunk2 = std::max(1, chunk1 / 4);
  if (tail < 0) tail = 0;  // automatic: no short-item phase (it measured no better)
  // at most 65535 samples per item: job indices (< 64 * chunk) stay below
  // 2^22, where the kernels' float-reciprocal division (div_small) is exact
  chunk1 = std::min({chunk1, spp, 65535});
  chunk2 = std::min(chunk2, 65535);
  tail = std::min(tail, spp);
  const int32_t spp1 = spp - tail;
  const int64_t grid_wpb = bvh ? GridShape<true>::waves : GridShape<false>::waves;
  int32_t nch1 = spp1 > 0 ? (spp1 + chunk1 - 1) / chunk1 : 0;
  if (ctx->chunk <= 0 && !persistent && !resident && spp1 >= grid_wpb) {
    // automatic grid schedule: exactly a multiple of the block's waves items
    // per tile, so a block's items share a tile and it flushes once
    // (block_flush).  chunk1 = ceil(spp1 / n1) can leave the last items of a
    // tile empty (spp1 = 5 on 4 waves: 2, 2, 1, 0 samples); an empty item's
    // wave takes no job and only joins the block's flush.
    int64_t n1 = (spp1 + chunk1 - 1) / chunk1;
    n1 = (n1 + grid_wpb - 1) / grid_wpb * grid_wpb;
    chunk1 = int32_t((spp1 + n1 - 1) / n1);
    nch1 = int32_t(n1);
  }
  chunk2 = std::min(chunk2, std::max(tail, 1));
  int32_t nch2 = tail > 0 ? (tail + chunk2 - 1) / chunk2 : 0;
  if (ctx->tail_chunk <= 0 && !persistent && !resident && tail >= grid_wpb) {
    // the short-item phase in a multiple of the block's waves items per tile
    // too, so its blocks also cover one tile each and flush once
    int64_t n2 = (nch2 + grid_wpb - 1) / grid_wpb * grid_wpb;
    chunk2 = int32_t((tail + n2 - 1) / n2);
    nch2 = int32_t(n2);
  }
  const int64_t items = tiles * (int64_t(nch1) + nch2);
  if (items > int64_t(INT32_MAX) - 8) return set_error(RT_EINVAL, "too many work items");
  RenderArgs a;
  a.cam = cam_f(cam);
  a.n = ctx->n;
  a.npairs = ctx->npairs;
  a.W = W; a.H = H; a.spp = spp; a.max_depth = max_depth; a.seed = seed;
  a.row0 = row0; a.row_step = row_step; a.nrows_valid = nvalid;
  a.tiles_x = tiles_x; a.n_items = int32_t(items);
  a.tiles = int32_t(tiles); a.spp1 = spp1; a.chunk1 = chunk1; a.nch1 = nch1; a.chunk2 = chunk2; a.nch2 = nch2;
  // block flush: every block's items are of one tile — both phases hold a
  // multiple of the block's waves items per tile
  a.block_flush = !persistent && !resident && nch1 % grid_wpb == 0 && nch2 % grid_wpb == 0 && ctx->block_flush;
  a.block_owns_tile = a.block_flush && !pass_accum && nch1 == grid_wpb && nch2 == 0 && ctx->block_owns;
  // the resident kernel: an item that covers all its tile's samples writes the floats
  if (resident) a.block_owns_tile = !pass_accum && nch1 == 1 && nch2 == 0 && ctx->block_owns;
  const bool chunked = pass_accum || nch1 + nch2 > 1;
  if (!ctx->probing) {
    const int32_t sched[8] = {TW, chunk1, nch1, nch2, a.block_flush + a.block_owns_tile, persistent ? 0 : 1,
                              resident ? 3 : (persistent ? 1 : 0), acc_kind == 3 ? 2 : (acc_kind == 5 ? 4 : acc_kind)};
    std::copy(sched, sched + 8, ctx->last_sched);
  }
  a.s_base = s_base;
  a.out_elems = uint64_t(nvalid) * uint64_t(W) * 3;
  const size_t n_valid_out = size_t(nvalid) * W * 3;
  if (chunked && !pass_accum && !a.block_owns_tile) {
    if (ctx->accum_cap < n_valid_out) {
      int rc = dev_alloc(&ctx->accum, n_valid_out);
      if (rc) { ctx->accum_cap = 0; return rc; }
      ctx->accum_cap = n_valid_out;
    }
  }
  // (after the allocation above, which may replace ctx->accum)
  unsigned long long *const accum = pass_accum ? pass_accum : ctx->accum;
  // host-side check of what the kernels will index: accumulator and output
  // hold the nvalid rows, every work item lies inside them
  if (chunked && !a.block_owns_tile && (!accum || (pass_accum ? ctx->pass_cap : ctx->accum_cap) < n_valid_out))
    return set_error(RT_EHIP, "internal: accumulator not allocated for %zu elements", n_valid_out);
  if ((!chunked || a.block_owns_tile) && !strip) return set_error(RT_EHIP, "internal: no output strip");
  if (int64_t(tiles_y) * TH < nvalid || int64_t(tiles_x) * TW < W || nch1 * int64_t(chunk1) < spp1 ||
      nch2 * int64_t(chunk2) < spp - spp1)
    return set_error(RT_EHIP, "internal: work items do not cover the image");
  a.acc = bvh ? accel_of(ctx, acc_kind) : Accel{nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, GridDesc{}};
  // cost-ordered dispatch: tiles sorted by the previous render's per-tile
  // world.hit counts (same layout), most expensive first, so the dispatch
  // tail is made of cheap items.  Changes the order of work only.
  a.tile_order = nullptr;
  a.tile_cost = nullptr;
  if (ctx->ordering == RT_ORDER_COST) {
    const int64_t key[6] = {W, H, row0, row_step, nvalid, TW};
    if (ctx->cost_cap < size_t(tiles)) {
      int rc;
      if ((rc = dev_alloc(&ctx->cost_prev, size_t(tiles))) || (rc = dev_alloc(&ctx->cost_cur, size_t(tiles))) ||
          (rc = dev_alloc(&ctx->cost_sorted, size_t(tiles))) || (rc = dev_alloc(&ctx->order, size_t(tiles))) ||
          (rc = dev_alloc(&ctx->iota, size_t(tiles)))) {
        ctx->cost_cap = 0;
        return rc;
      }
      std::vector<int32_t> io(static_cast<size_t>(tiles));
      for (int64_t t = 0; t < tiles; ++t) io[size_t(t)] = int32_t(t);
      HIP_TRY(hipMemcpy(ctx->iota, io.data(), io.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      ctx->cost_cap = size_t(tiles);
      ctx->cost_valid = false;
      size_t need = 0;
      HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, need, ctx->cost_prev, ctx->cost_sorted, ctx->iota,
                                                           ctx->order, int(tiles)));
      if (need > ctx->sort_tmp_bytes) {
        if (ctx->sort_tmp) (void)hipFree(ctx->sort_tmp);
        ctx->sort_tmp = nullptr;
        HIP_TRY(hipMalloc(&ctx->sort_tmp, need));
        ctx->sort_tmp_bytes = need;
      }
    }
    const bool have_map = ctx->cost_valid && std::equal(key, key + 6, ctx->cost_key);
    // Probe: 1 sample per pixel, paths cut at depth 8, rendered into the
    // output strip (overwritten by this render) counts world.hit per tile,
    // under 1/500 of the render's work; the render then dispatches by those counts.
    if (!ctx->probing && strip && !pass_accum && spp >= 16 &&
        (ctx->probe_mode == 2 || (ctx->probe_mode == 1 && !have_map))) {
      ctx->probing = true;
      const int32_t pspp = ctx->probe_spp > 0 ? std::min(ctx->probe_spp, spp) : 1;
      const int32_t pdepth = std::min(ctx->probe_depth > 0 ? ctx->probe_depth : 8, max_depth);
      const int rc = render_rows_impl(ctx, cam, W, H, pspp, pdepth, seed, row0, row_step, nrows, strip,
                                      st, s_base, nullptr);
      ctx->probing = false;
      if (rc) return rc;
      HIP_TRY(hipMemsetAsync(ctx->segments, 0, 8 * sizeof(unsigned long long), st));  // count this render only
    }
    if (ctx->cost_valid && std::equal(key, key + 6, ctx->cost_key)) {
      size_t bytes = ctx->sort_tmp_bytes;
      HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(ctx->sort_tmp, bytes, ctx->cost_prev, ctx->cost_sorted,
                                                           ctx->iota, ctx->order, int(tiles), 0, 32, st));
      a.tile_order = ctx->order;
    }
    HIP_TRY(hipMemsetAsync(ctx->cost_cur, 0, size_t(tiles) * sizeof(unsigned), st));
    a.tile_cost = ctx->cost_cur;
    std::swap(ctx->cost_prev, ctx->cost_cur);  // this launch's counts order the next one
    std::copy(key, key + 6, ctx->cost_key);
    ctx->cost_valid = true;
  }
  // (cleared here, after the cost probe, which may render into the same
  // accumulator)
  if (chunked && !pass_accum && !a.block_owns_tile)
    HIP_TRY(hipMemsetAsync(ctx->accum, 0, n_valid_out * sizeof(unsigned long long), st));
  dim3 grid;
  if (resident) {
#if RTMI_EXPERIMENTAL
    // CU-resident blocks; waves past the first grid's take items from the counter
    HIP_TRY(hipMemsetAsync(ctx->counter, 0, sizeof(unsigned), st));
    RenderArgs b = a;
    const size_t lds = res_lds_bytes(a.acc, acc_kind, &b.acc_off);
    const int64_t rblocks = res_resident_blocks(ctx, lds);
    grid = dim3(unsigned(std::min<int64_t>((items + kResWaves - 1) / kResWaves, rblocks)));
    switch (TW) {
      case 8: launch_resident<8>(acc_kind, grid, lds, st, ctx, b, accum, strip); break;
      default: launch_resident<16>(acc_kind, grid, lds, st, ctx, b, accum, strip); break;
    }
#endif
  } else if (persistent) {
    // a resident grid of waves pulling items from a global counter
    HIP_TRY(hipMemsetAsync(ctx->counter, 0, sizeof(unsigned), st));
    const int64_t pw = kWavesPerBlock;
    const int64_t waves = std::min<int64_t>(items, int64_t(ctx->resident_blocks) * pw);
    grid = dim3(unsigned((waves + pw - 1) / pw));
  } else {
    const int64_t wpb = bvh ? GridShape<true>::waves : GridShape<false>::waves;
    grid = dim3(unsigned((items + wpb - 1) / wpb));
  }
  if (!resident) switch (TW) {
    case 8: launch_shape<8>(persistent, acc_kind, chunked, grid, st, ctx, a, accum, strip); break;
    case 16: launch_shape<16>(persistent, acc_kind, chunked, grid, st, ctx, a, accum, strip); break;
    case 32: launch_shape<32>(persistent, acc_kind, chunked, grid, st, ctx, a, accum, strip); break;
    default: launch_shape<64>(persistent, acc_kind, chunked, grid, st, ctx, a, accum, strip); break;
  }
  HIP_TRY(hipGetLastError());
  if (chunked && !pass_accum && !a.block_owns_tile) {
    hipLaunchKernelGGL(finalize_kernel, dim3(unsigned((n_valid_out + 255) / 256)), dim3(256), 0, st, ctx->accum,
                       strip, n_valid_out);
    HIP_TRY(hipGetLastError());
  }
  return RT_OK;
}

}  // namespace

RTMI_EXPORT int rt_render_rows(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                               int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows,
                               float *dev_strip, void *stream) {
  int rc = check_render_args(ctx, cam, W, H, spp, max_depth);
  if (rc) return rc;
  if (row0 < 0 || row_step < 1 || nrows < 0 || (nrows > 0 && !dev_strip))
    return set_error(RT_EINVAL, "rt_render_rows: bad row set");
  DeviceGuard guard(ctx->device);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  return render_rows_impl(ctx, cam, W, H, spp, max_depth, seed, row0, row_step, nrows, dev_strip, st);
}

// ---------------------------------------------------------------------------
// progressive accumulation
// ---------------------------------------------------------------------------
// The accumulator holds the fixed-point sums (2^-32, int64) of the passes
// so far; integer addition makes any split of [0, spp) into passes give the
// same sums, bit for bit, as one rt_render of spp samples.
RTMI_EXPORT int rt_accum_reset(rt_ctx *ctx, int32_t W, int32_t nrows) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (W < 1 || nrows < 0) return set_error(RT_EINVAL, "rt_accum_reset: bad size %dx%d", W, nrows);
  DeviceGuard guard(ctx->device);
  const size_t n = size_t(W) * size_t(nrows) * 3;
  if (ctx->pass_cap < n) {
    int rc = dev_alloc(&ctx->pass_accum, std::max<size_t>(n, 1));
    if (rc) { ctx->pass_cap = 0; return rc; }
    ctx->pass_cap = n;
  }
  ctx->pass_W = W;
  ctx->pass_rows = nrows;
  ctx->pass_spp = 0;
  if (ctx->last_stream) HIP_TRY(hipStreamSynchronize(ctx->last_stream));  // no pass still adding
  if (n) HIP_TRY(hipMemsetAsync(ctx->pass_accum, 0, n * sizeof(unsigned long long), ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RT_OK;
}

RTMI_EXPORT int rt_render_pass(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t s_begin,
                               int32_t s_count, int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                               int32_t nrows, void *stream) {
  int rc = check_render_args(ctx, cam, W, H, std::max(s_count, 1), max_depth);
  if (rc) return rc;
  if (s_begin < 0 || s_count < 0 || int64_t(s_begin) + s_count > INT32_MAX)
    return set_error(RT_EINVAL, "rt_render_pass: bad sample range [%d, +%d)", s_begin, s_count);
  if (row0 < 0 || row_step < 1 || nrows < 0) return set_error(RT_EINVAL, "rt_render_pass: bad row set");
  if (!ctx->pass_accum || W != ctx->pass_W || nrows != ctx->pass_rows)
    return set_error(RT_EINVAL, "rt_render_pass: accumulator is not %dx%d (call rt_accum_reset)", W, nrows);
  DeviceGuard guard(ctx->device);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if ((rc = render_rows_impl(ctx, cam, W, H, s_count, max_depth, seed, row0, row_step, nrows, nullptr, st, s_begin,
                             ctx->pass_accum)))
    return rc;
  ctx->pass_spp += s_count;
  return RT_OK;
}

RTMI_EXPORT int rt_accum_resolve(rt_ctx *ctx, float *dev_sum, float *host_sum, void *stream) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  if (!ctx->pass_accum) return set_error(RT_EINVAL, "rt_accum_resolve: no accumulator");
  if (!dev_sum && !host_sum) return set_error(RT_EINVAL, "rt_accum_resolve: no output");
  DeviceGuard guard(ctx->device);
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (ctx->last_stream && ctx->last_stream != st) HIP_TRY(hipStreamWaitEvent(st, ctx->last_done, 0));
  const size_t n = size_t(ctx->pass_W) * size_t(ctx->pass_rows) * 3;
  float *out = dev_sum;
  if (!out) {
    if (ctx->scratch_cap < n) {
      int rc = dev_alloc(&ctx->scratch, n);
      if (rc) { ctx->scratch_cap = 0; return rc; }
      ctx->scratch_cap = n;
    }
    out = ctx->scratch;
  }
  if (n) {
    hipLaunchKernelGGL(finalize_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, ctx->pass_accum, out, n);
    HIP_TRY(hipGetLastError());
  }
  if (host_sum) {
    if (n) HIP_TRY(hipMemcpyAsync(host_sum, out, n * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  return RT_OK;
}

// Checkpoint / resume: the raw fixed-point accumulator (W*nrows*3 int64) and
// the number of samples it holds.
RTMI_EXPORT int rt_accum_export(rt_ctx *ctx, int64_t *host, size_t n, int32_t *spp_done) {
  if (!ctx || !host) return set_error(RT_EINVAL, "null argument");
  const size_t want = size_t(ctx->pass_W) * size_t(ctx->pass_rows) * 3;
  if (!ctx->pass_accum || n != want) return set_error(RT_EINVAL, "rt_accum_export: size %zu, accumulator %zu", n, want);
  DeviceGuard guard(ctx->device);
  HIP_TRY(hipStreamSynchronize(ctx->last_stream ? ctx->last_stream : ctx->stream));
  HIP_TRY(hipMemcpy(host, ctx->pass_accum, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (spp_done) *spp_done = ctx->pass_spp;
  return RT_OK;
}

RTMI_EXPORT int rt_accum_import(rt_ctx *ctx, const int64_t *host, size_t n, int32_t spp_done) {
  if (!ctx || !host) return set_error(RT_EINVAL, "null argument");
  const size_t want = size_t(ctx->pass_W) * size_t(ctx->pass_rows) * 3;
  if (!ctx->pass_accum || n != want)
    return set_error(RT_EINVAL, "rt_accum_import: size %zu, accumulator %zu (call rt_accum_reset)", n, want);
  if (spp_done < 0) return set_error(RT_EINVAL, "rt_accum_import: negative sample count");
  DeviceGuard guard(ctx->device);
  if (ctx->last_stream) HIP_TRY(hipStreamSynchronize(ctx->last_stream));
  HIP_TRY(hipMemcpy(ctx->pass_accum, host, n * sizeof(int64_t), hipMemcpyHostToDevice));
  ctx->pass_spp = spp_done;
  return RT_OK;
}

namespace {
// Checkpoint file (little-endian): "RTMIACC1", int32 W H row0 row_step nrows
// spp_done max_depth 0, u64 seed, u64 FNV-1a of the scene arrays, u64 FNV-1a
// of the camera, then the int64 accumulator [nrows][W][3].
constexpr char kCkptMagic[8] = {'R', 'T', 'M', 'I', 'A', 'C', 'C', '1'};
struct CkptHeader {
  char magic[8];
  int32_t W, H, row0, row_step, nrows, spp_done, max_depth, zero;
  uint64_t seed, scene_hash, camera_hash;
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header layout");

uint64_t fnv1a(uint64_t h, const void *p, size_t n) {
  const unsigned char *b = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}
uint64_t scene_hash(const rt_scene *s) {
  uint64_t h = 14695981039346656037ull;
  h = fnv1a(h, &s->n, sizeof s->n);
  h = fnv1a(h, s->center_radius, sizeof(double) * 4 * size_t(s->n));
  h = fnv1a(h, s->mat_kind, sizeof(int32_t) * size_t(s->n));
  return fnv1a(h, s->mat_params, sizeof(double) * 4 * size_t(s->n));
}
uint64_t camera_hash(const rt_camera *c) { return fnv1a(14695981039346656037ull, c, sizeof *c); }
}  // namespace

RTMI_EXPORT int rt_accum_save(rt_ctx *ctx, const char *path, const rt_scene *scene, const rt_camera *cam, int32_t H,
                              int32_t row0, int32_t row_step, int32_t max_depth, uint64_t seed) {
  if (!ctx || !path || !scene || !cam) return set_error(RT_EINVAL, "rt_accum_save: null argument");
  if (!ctx->pass_accum) return set_error(RT_EINVAL, "rt_accum_save: no accumulator");
  const size_t n = size_t(ctx->pass_W) * size_t(ctx->pass_rows) * 3;
  std::vector<int64_t> raw(n);
  int32_t done = 0;
  if (int rc = rt_accum_export(ctx, raw.data(), n, &done)) return rc;
  CkptHeader h{};
  std::memcpy(h.magic, kCkptMagic, 8);
  h.W = ctx->pass_W; h.H = H; h.row0 = row0; h.row_step = row_step; h.nrows = ctx->pass_rows;
  h.spp_done = done; h.max_depth = max_depth; h.zero = 0;
  h.seed = seed; h.scene_hash = scene_hash(scene); h.camera_hash = camera_hash(cam);
  const std::string tmp = std::string(path) + ".tmp";
  FILE *f = std::fopen(tmp.c_str(), "wb");
  if (!f) return set_error(RT_EIO, "rt_accum_save: cannot open %s", tmp.c_str());
  bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(raw.data(), sizeof(int64_t), n, f) == n;
  if (std::fclose(f) != 0) ok = false;
  if (!ok || std::rename(tmp.c_str(), path) != 0) return set_error(RT_EIO, "rt_accum_save: write to %s failed", path);
  return RT_OK;
}

RTMI_EXPORT int rt_accum_load(rt_ctx *ctx, const char *path, const rt_scene *scene, const rt_camera *cam, int32_t W,
                              int32_t H, int32_t row0, int32_t row_step, int32_t nrows, int32_t max_depth,
                              uint64_t seed, int32_t *spp_done) {
  if (!ctx || !path || !scene || !cam || !spp_done) return set_error(RT_EINVAL, "rt_accum_load: null argument");
  FILE *f = std::fopen(path, "rb");
  if (!f) return set_error(RT_EIO, "rt_accum_load: cannot open %s", path);
  CkptHeader h{};
  const bool hdr = std::fread(&h, sizeof h, 1, f) == 1;
  if (!hdr || std::memcmp(h.magic, kCkptMagic, 8) != 0) {
    std::fclose(f);
    return set_error(RT_EIO, "rt_accum_load: %s is not a checkpoint", path);
  }
  if (h.W != W || h.H != H || h.row0 != row0 || h.row_step != row_step || h.nrows != nrows || h.max_depth != max_depth ||
      h.seed != seed || h.scene_hash != scene_hash(scene) || h.camera_hash != camera_hash(cam)) {
    std::fclose(f);
    return set_error(RT_EINVAL, "rt_accum_load: %s was made for another render (size, rows, depth, seed, scene or camera)",
                     path);
  }
  const size_t n = size_t(W) * size_t(nrows) * 3;
  std::vector<int64_t> raw(n);
  const bool body = std::fread(raw.data(), sizeof(int64_t), n, f) == n;
  std::fclose(f);
  if (!body) return set_error(RT_EIO, "rt_accum_load: %s is truncated", path);
  if (int rc = rt_accum_reset(ctx, W, nrows)) return rc;
  if (int rc = rt_accum_import(ctx, raw.data(), n, h.spp_done)) return rc;
  *spp_done = h.spp_done;
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_synchronize(rt_ctx *ctx) {
  if (!ctx) return set_error(RT_EINVAL, "null ctx");
  DeviceGuard guard(ctx->device);
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  // (and the stream of the last render, when it ran on a caller's stream)
  if (ctx->last_stream && ctx->last_stream != ctx->stream) HIP_TRY(hipStreamSynchronize(ctx->last_stream));
  return RT_OK;
}

RTMI_EXPORT int rt_render(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp, int32_t max_depth,
                          uint64_t seed, float *sum) {
  int rc = check_render_args(ctx, cam, W, H, spp, max_depth);
  if (rc) return rc;
  if (!sum) return set_error(RT_EINVAL, "null output");
  DeviceGuard guard(ctx->device);
  const size_t n = size_t(W) * H * 3;
  if (ctx->scratch_cap < n) {
    if ((rc = dev_alloc(&ctx->scratch, n))) { ctx->scratch_cap = 0; return rc; }
    ctx->scratch_cap = n;
  }
  if ((rc = render_rows_impl(ctx, cam, W, H, spp, max_depth, seed, 0, 1, H, ctx->scratch, ctx->stream))) return rc;
  HIP_TRY(hipMemcpyAsync(sum, ctx->scratch, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RT_OK;
}

RTMI_EXPORT int rt_replay_worker(rt_ctx *ctx, const rt_camera *cam, int32_t W, int32_t H, int32_t spp,
                                 int32_t max_depth, int32_t n_jobs, const int32_t *job_ranges, const int32_t *streams,
                                 const int64_t *stream_offsets, double *host_sums, int64_t *draws_used) {
  int rc = check_render_args(ctx, cam, W, H, spp, max_depth);
  if (rc) return rc;
  if (max_depth > kMaxReplayDepth) return set_error(RT_EINVAL, "replay max_depth must be <= %d", kMaxReplayDepth);
  if (n_jobs <= 0 || !job_ranges || !stream_offsets || !host_sums || !draws_used)
    return set_error(RT_EINVAL, "rt_replay_worker: bad argument");
  std::vector<int64_t> out_offs(n_jobs + 1, 0);
  for (int k = 0; k < n_jobs; k++) {
    const int s = job_ranges[2 * k], e = job_ranges[2 * k + 1];
    if (s < 0 || e < s || int64_t(e) > int64_t(W) * H) return set_error(RT_EINVAL, "job %d: bad range", k);
    if (stream_offsets[k + 1] < stream_offsets[k]) return set_error(RT_EINVAL, "job %d: bad stream offsets", k);
    out_offs[k + 1] = out_offs[k] + 3 * int64_t(e - s);
  }
  const int64_t n_stream = stream_offsets[n_jobs];
  DeviceGuard guard(ctx->device);
  int32_t *d_ranges = nullptr, *d_streams = nullptr;
  int64_t *d_offs = nullptr, *d_oo = nullptr, *d_used = nullptr;
  double *d_out = nullptr;
  auto cleanup = [&]() {
    for (void *p : {(void *)d_ranges, (void *)d_streams, (void *)d_offs, (void *)d_oo, (void *)d_used, (void *)d_out})
      if (p) (void)hipFree(p);
  };
  if ((rc = dev_alloc(&d_ranges, 2 * size_t(n_jobs))) || (rc = dev_alloc(&d_streams, size_t(n_stream))) ||
      (rc = dev_alloc(&d_offs, size_t(n_jobs) + 1)) || (rc = dev_alloc(&d_oo, size_t(n_jobs) + 1)) ||
      (rc = dev_alloc(&d_used, size_t(n_jobs))) || (rc = dev_alloc(&d_out, size_t(out_offs[n_jobs])))) {
    cleanup();
    return rc;
  }
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  chk(hipMemcpy(d_ranges, job_ranges, 2 * size_t(n_jobs) * sizeof(int32_t), hipMemcpyHostToDevice));
  if (n_stream > 0 && streams) chk(hipMemcpy(d_streams, streams, size_t(n_stream) * sizeof(int32_t), hipMemcpyHostToDevice));
  chk(hipMemcpy(d_offs, stream_offsets, (size_t(n_jobs) + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  chk(hipMemcpy(d_oo, out_offs.data(), (size_t(n_jobs) + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  ReplayArgs a;
  a.cam = cam_d(cam);
  a.n = ctx->n; a.W = W; a.H = H; a.spp = spp; a.max_depth = max_depth; a.n_jobs = n_jobs;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(replay_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, ctx->stream, ctx->geom64, ctx->sh064,
                       ctx->sh164, a, d_ranges, d_streams, d_offs, d_oo, d_out, d_used);
    chk(hipGetLastError());
    chk(hipStreamSynchronize(ctx->stream));
    chk(hipMemcpy(host_sums, d_out, size_t(out_offs[n_jobs]) * sizeof(double), hipMemcpyDeviceToHost));
    chk(hipMemcpy(draws_used, d_used, size_t(n_jobs) * sizeof(int64_t), hipMemcpyDeviceToHost));
  }
  cleanup();
  if (e != hipSuccess) return set_error(RT_EHIP, "rt_replay_worker: %s", hipGetErrorString(e));
  for (int k = 0; k < n_jobs; k++)
    if (draws_used[k] < 0) return set_error(RT_ESTREAM, "job %d ran out of stream values", k);
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_last_schedule(rt_ctx *ctx, int32_t *out8) {
  if (!ctx || !out8) return set_error(RT_EINVAL, "null");
  std::copy(ctx->last_sched, ctx->last_sched + 8, out8);
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_last_segments(rt_ctx *ctx, uint64_t *segments) {
  if (!ctx || !segments) return set_error(RT_EINVAL, "null argument");
  DeviceGuard guard(ctx->device);
  hipStream_t st = ctx->last_stream ? ctx->last_stream : ctx->stream;
  unsigned long long v = 0;
  HIP_TRY(hipMemcpyAsync(&v, ctx->segments, sizeof v, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *segments = v;
  return RT_OK;
}

// Debug counters of the last render (RTMI_STATS builds only; zeros otherwise):
// out[0] = world.hit calls, out[1] = sphere groups tested (per wave),
// out[2] = groups where some lane had a candidate, out[3] = candidate resolves
// (lane), out[4] = candidate spheres resolved (wave); out has 8 slots.
// Per-wave trace of the renders since the last call (RTMI_TRACE builds; 0
// lines otherwise): 4 u64 per wave, see RTMI_TRACE_END.  Returns the count.
RTMI_EXPORT int rt_ctx_debug_trace(rt_ctx *ctx, uint64_t *out, int32_t cap) {
  if (!ctx || !out) return set_error(RT_EINVAL, "null argument");
#if RTMI_TRACE
  DeviceGuard guard(ctx->device);
  HIP_TRY(hipDeviceSynchronize());
  unsigned n = 0;
  HIP_TRY(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_trace_n), sizeof n));
  n = std::min<unsigned>(std::min<unsigned>(n, kTraceCap), unsigned(std::max(cap, 0)));
  if (n) HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), size_t(n) * 4 * sizeof(uint64_t)));
  const unsigned zero = 0;
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_trace_n), &zero, sizeof zero));
  return int(n);
#else
  (void)cap;
  return 0;
#endif
}

// Validation: brute-force and accelerated closest hits of n rays (host
// arrays): rays[6n] = o.xyz d.xyz; idx[2n] = {brute, accelerated} sphere
// index (-1 miss); t[2n] likewise.  The accelerated search is the context's
// RT_ACCEL_GRID when selected, else the BVH.  Not part of the render path.
RTMI_EXPORT int rt_ctx_debug_hits(rt_ctx *ctx, const float *rays, int32_t n, int32_t *idx, float *t) {
  if (!ctx || !rays || !idx || !t || n < 0) return set_error(RT_EINVAL, "rt_ctx_debug_hits: bad argument");
  if (n == 0) return RT_OK;
  if (ctx->n <= 0) return set_error(RT_EINVAL, "no scene");
  DeviceGuard guard(ctx->device);
  float *d_rays = nullptr, *d_t = nullptr;
  int32_t *d_idx = nullptr;
  int rc;
  if ((rc = dev_alloc(&d_rays, size_t(n) * 6)) || (rc = dev_alloc(&d_idx, size_t(n) * 2)) ||
      (rc = dev_alloc(&d_t, size_t(n) * 2)))
    return rc;
  HIP_TRY(hipMemcpy(d_rays, rays, size_t(n) * 6 * sizeof(float), hipMemcpyHostToDevice));
  // the walk the renders use, by render_rows_impl's rule (3: the one-layer
  // grid walk; +2: walked in global memory; 1: the BVH, also where the grid
  // setting has no grid, e.g. over 65 535 spheres)
  const int kind = ctx->accel == RT_ACCEL_GRID && ctx->grid_ok
                       ? (ctx->grid.n[1] == 1 ? 3 : 2) + (ctx->grid_global ? 2 : 0)
                       : (ctx->accel != RT_ACCEL_NONE && ctx->nnodes > 0 ? 1 : 0);
  if (kind == 0) {
    (void)hipFree(d_rays); (void)hipFree(d_idx); (void)hipFree(d_t);
    return set_error(RT_EUNSUPPORTED, "rt_ctx_debug_hits: brute force only for this scene and setting (no structure)");
  }
  const Accel acc = accel_of(ctx, kind);
  const size_t lds = accel_lds_bytes(acc, kind);
  if (kind == 1)
    hipLaunchKernelGGL(debug_hit_kernel<1>, dim3(unsigned((n + 255) / 256)), dim3(256), lds, ctx->stream, ctx->pairs,
                       ctx->npairs, acc, d_rays, n, d_idx, d_t);
  else if (kind == 2)
    hipLaunchKernelGGL(debug_hit_kernel<2>, dim3(unsigned((n + 255) / 256)), dim3(256), lds, ctx->stream, ctx->pairs,
                       ctx->npairs, acc, d_rays, n, d_idx, d_t);
  else if (kind == 3)
    hipLaunchKernelGGL(debug_hit_kernel<3>, dim3(unsigned((n + 255) / 256)), dim3(256), lds, ctx->stream, ctx->pairs,
                       ctx->npairs, acc, d_rays, n, d_idx, d_t);
  else if (kind == 4)
    hipLaunchKernelGGL(debug_hit_kernel<4>, dim3(unsigned((n + 255) / 256)), dim3(256), lds, ctx->stream, ctx->pairs,
                       ctx->npairs, acc, d_rays, n, d_idx, d_t);
  else
    hipLaunchKernelGGL(debug_hit_kernel<5>, dim3(unsigned((n + 255) / 256)), dim3(256), lds, ctx->stream, ctx->pairs,
                       ctx->npairs, acc, d_rays, n, d_idx, d_t);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipMemcpy(idx, d_idx, size_t(n) * 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(t, d_t, size_t(n) * 2 * sizeof(float), hipMemcpyDeviceToHost));
  (void)hipFree(d_rays);
  (void)hipFree(d_idx);
  (void)hipFree(d_t);
  return RT_OK;
}

// Exhaustive check of the fast correctly rounded float routines (rtmi_path.h
// sqrt_cr / rcp_cr) against the compiler's IEEE lowering: every one of the
// 2^32 bit patterns (NaN == NaN whatever the payload).  out[0] mismatches,
// out[1] the smallest mismatching input, out[2] / out[3] the two results
// there.  Diagnostic (tests), not part of the render path.
__global__ void exact_math_kernel(int32_t which, unsigned long long *res) {
  const uint32_t base = (uint32_t(blockIdx.x) * blockDim.x + threadIdx.x) << 8;
  unsigned bad = 0;
  uint32_t first = 0xFFFFFFFFu, got_first = 0, want_first = 0;
  for (uint32_t k = 0; k < 256; ++k) {
    const uint32_t bits = base + k;
    const float x = __uint_as_float(bits);
    const float got = which == 0 ? sqrt_cr(x) : rcp_cr(x);
    const float want = which == 0 ? __builtin_sqrtf(x) : 1.0f / x;
    const bool same = __float_as_uint(got) == __float_as_uint(want) || (got != got && want != want);
    if (!same) {
      ++bad;
      if (bits < first) { first = bits; got_first = __float_as_uint(got); want_first = __float_as_uint(want); }
    }
  }
  if (bad) {
    atomicAdd(&res[0], (unsigned long long)bad);
    const unsigned long long old = atomicMin(&res[1], (unsigned long long)first);
    if (first < old) { res[2] = got_first; res[3] = want_first; }  // (racy only between mismatching threads)
  }
}

RTMI_EXPORT int rt_debug_exact_math(int32_t which, uint64_t *out) {
  if (!out || which < 0 || which > 1) return set_error(RT_EINVAL, "rt_debug_exact_math: bad argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return set_error(RT_ENODEVICE, "no GPU");
  unsigned long long *d = nullptr;
  int rc;
  if ((rc = dev_alloc(&d, 4))) return rc;
  const unsigned long long init[4] = {0, ~0ull, 0, 0};
  HIP_TRY(hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(exact_math_kernel, dim3(1u << 16), dim3(256), 0, nullptr, which, d);  // 2^24 threads x 256
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  unsigned long long v[4];
  HIP_TRY(hipMemcpy(v, d, sizeof v, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  for (int i = 0; i < 4; i++) out[i] = v[i];
  return RT_OK;
}

RTMI_EXPORT int rt_ctx_debug_counters(rt_ctx *ctx, uint64_t *out) {
  if (!ctx || !out) return set_error(RT_EINVAL, "null argument");
  DeviceGuard guard(ctx->device);
  hipStream_t st = ctx->last_stream ? ctx->last_stream : ctx->stream;
  unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(v, ctx->segments, sizeof v, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (int i = 0; i < 8; i++) out[i] = v[i];
  return RT_OK;
}
