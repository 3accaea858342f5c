// rtmi_path.h — device-side path tracing for librtmi: numeric policy, RNG,
// camera ray, ray-sphere loops, materials (the reference's L0-L4 layers:
// vec3.h, ray.h, camera.h, sphere.h, hittable_list.h, material.h,
// main.cpp:57-83).  Included by rtmi_device.hip (the kernels) and by
// tools/loopbench.hip (the sphere-loop microbenchmark).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "../../include/rtmi.h"

#ifndef RTMI_STATS
#define RTMI_STATS 0
#endif

namespace rtmi {


constexpr int kGeomPad = 16;  // zero spheres after the scene's geom records (padding)

// ---------------------------------------------------------------------------
// numeric policy
// ---------------------------------------------------------------------------
template <class R> struct V3 { R x, y, z; };
template <class R> __host__ __device__ __forceinline__ V3<R> mk(R x, R y, R z) { return V3<R>{x, y, z}; }

template <bool F> __device__ __forceinline__ float madd(float a, float b, float c) {
  if constexpr (F) return __builtin_fmaf(a, b, c);
  else return a * b + c;
}
template <bool F> __device__ __forceinline__ double madd(double a, double b, double c) {
  if constexpr (F) return __builtin_fma(a, b, c);
  else return a * b + c;
}
// Correctly rounded float sqrt and reciprocal in fewer instructions than the
// compiler's IEEE lowering (~16 and ~10 VALU: denormal scaling, class checks,
// v_div_scale / v_div_fmas / v_div_fixup), bit-identical to it for EVERY one
// of the 2^32 inputs (rt_debug_exact_math checks all of them on the GPU:
// tests/test_gpu_parity.py::test_exact_math_exhaustive).
//  sqrt: the hardware v_sqrt_f32 (within 1 ulp), then the neighbour below or
//  above when the exact residual x - s'*s says the true root lies past the
//  midpoint (+inf passes through: its residuals are NaN); inputs below 2^-96
//  keep the IEEE lowering.
//  reciprocal: v_rcp_f32, then one Newton step with exact fma residual; the
//  ranges where 1/x or x lies outside the normal range keep the IEEE
//  division (a branch no realistic scene takes).
// (The out-of-range inputs take the IEEE form behind a wave-uniform branch on
// their ballot: the common path pays one compare and a scalar branch, not an
// exec-mask save/restore — DESIGN.md §4.5.)
__device__ __forceinline__ float sqrt_cr(float x) {
  // below 2^-96 (zero, denormals — which v_sqrt_f32 flushes — negatives,
  // NaN) the residuals would underflow: the IEEE lowering
  const bool slow = !(x >= 0x1p-96f);
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
  float r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
  r = __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    if (slow) r = __builtin_sqrtf(x);
  }
  return r;
}
__device__ __forceinline__ float rcp_cr(float x) {
  const float ax = __builtin_fabsf(x);
  const bool slow = !(ax >= 0x1p-125f && ax <= 0x1p+125f);  // zero, denormal, huge, inf, NaN
  const float r0 = __builtin_amdgcn_rcpf(x);
  float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    if (slow) r = 1.0f / x;
  }
  return r;
}
__device__ __forceinline__ float dsqrt(float x) { return sqrt_cr(x); }
__device__ __forceinline__ float drcp(float x) { return rcp_cr(x); }
__device__ __forceinline__ double dsqrt(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ double drcp(double x) { return 1.0 / x; }
__device__ __forceinline__ float dfabs(float x) { return __builtin_fabsf(x); }
__device__ __forceinline__ double dfabs(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float dfmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double dfmin(double a, double b) { return __builtin_fmin(a, b); }
// pow((1-cosine), 5) material.h:95: the exact path uses the library pow; the
// fast path multiplies (x^2)^2 * x (the CPU restatement does the same).
__device__ __forceinline__ float pow5(float x) { float x2 = x * x; float x4 = x2 * x2; return x4 * x; }
__device__ __forceinline__ double pow5(double x) { return pow(x, 5.0); }

// dot vec3.h:77-79
template <bool F, class R> __device__ __forceinline__ R dot(V3<R> a, V3<R> b) {
  return madd<F>(a.z, b.z, madd<F>(a.y, b.y, a.x * b.x));
}
template <class R> __device__ __forceinline__ V3<R> scale(R t, V3<R> v) { return mk(t * v.x, t * v.y, t * v.z); }
// unit_vector vec3.h:101 (operator/ is (1/t)*v, vec3.h:89)
template <bool F, class R> __device__ __forceinline__ V3<R> unit(V3<R> v) {
  return scale(drcp(dsqrt(dot<F>(v, v))), v);
}
// reflect vec3.h:114
template <bool F, class R> __device__ __forceinline__ V3<R> reflect(V3<R> v, V3<R> n) {
  const R k = R(2) * dot<F>(v, n);
  return mk(madd<F>(-k, n.x, v.x), madd<F>(-k, n.y, v.y), madd<F>(-k, n.z, v.z));
}
// refract vec3.h:116-121 (cos_theta identical to the caller's, material.h:72)
template <bool F, class R> __device__ __forceinline__ V3<R> refract(V3<R> uv, V3<R> n, R eta, R cos_theta) {
  V3<R> perp = mk(eta * madd<F>(cos_theta, n.x, uv.x), eta * madd<F>(cos_theta, n.y, uv.y),
                  eta * madd<F>(cos_theta, n.z, uv.z));
  const R s = dsqrt(dfabs(R(1) - dot<F>(perp, perp)));
  return mk(madd<F>(-s, n.x, perp.x), madd<F>(-s, n.y, perp.y), madd<F>(-s, n.z, perp.z));
}
// dielectric::reflectance material.h:91-96 (Schlick)
template <bool F, class R> __device__ __forceinline__ R reflectance(R cosine, R ref_idx) {
  R r0 = (R(1) - ref_idx) / (R(1) + ref_idx);
  r0 = r0 * r0;
  return madd<F>(R(1) - r0, pow5(R(1) - cosine), r0);
}
// near_zero vec3.h:53-57 — keeps the reference's fabs(e[0] < s) slip
template <class R> __device__ __forceinline__ bool near_zero(V3<R> v) {
  const R s = R(1e-8);
  return (v.x < s) && (dfabs(v.y) < s) && (dfabs(v.z) < s);
}

// ---------------------------------------------------------------------------
// RNG
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
// xoroshiro128+ (a=24, b=16, c=37), state from splitmix64 finalisers of the
// key (seed, pixel, sample): a counter-based stream per camera sample.
struct Xoro {
  uint64_t s0, s1;
  __device__ __forceinline__ void init(uint64_t seed, uint64_t pixel, uint32_t sample) {
    // splitmix64 with the (pixel, sample) key as its counter (the oracle's
    // xo_init is the same)
    const uint64_t key = (pixel << 24) | uint64_t(sample);
    s0 = mix64(seed ^ (key * 0x9E3779B97F4A7C15ULL));
    s1 = mix64(s0 + 0x9E3779B97F4A7C15ULL);
  }
  __device__ __forceinline__ uint64_t next() {
    const uint64_t a = s0, r = s0 + s1;
    uint64_t b = s1 ^ a;
    s0 = ((a << 24) | (a >> 40)) ^ b ^ (b << 16);
    s1 = (b << 37) | (b >> 27);
    return r;
  }
  // top 24 bits: uniform on [0,1) exactly representable in float
  // (32-bit extraction spelled out: the compiler otherwise emits a 64-bit
  // integer -> float conversion for some uses)
  __device__ __forceinline__ float uni() { return float(uint32_t(next() >> 32) >> 8) * 0x1p-24f; }
  // two uniforms from one step: bits 63..40 and 39..16
  __device__ __forceinline__ void pair(float &u, float &v) {
    const uint64_t r = next();
    const uint32_t hi = uint32_t(r >> 32), lo = uint32_t(r);
    u = float(hi >> 8) * 0x1p-24f;
    v = float(((hi & 0xFFu) << 16) | (lo >> 16)) * 0x1p-24f;
  }
};

// cos and sin of 2*pi*v, v in [0,1) a multiple of 2^-24: exact quadrant
// reduction, then Cephes' sinf/cosf polynomials on [-pi/4, pi/4] with
// explicit fma — the oracle's sincos2pi, operation for operation.
__device__ __forceinline__ void sincos2pi(float v, float &c, float &s) {
  const float t = v * 4.0f;
  const int k = int(t + 0.5f);
  const float x = (t - float(k)) * 1.57079637f;
  const float x2 = x * x;
  float p = __builtin_fmaf(x2, -1.9515295891e-4f, 8.3321608736e-3f);
  p = __builtin_fmaf(x2, p, -1.6666654611e-1f);
  const float sn = __builtin_fmaf(x * x2, p, x);
  float q = __builtin_fmaf(x2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  q = __builtin_fmaf(x2, q, 4.166664568298827e-2f);
  const float cs = __builtin_fmaf(x2 * x2, q, __builtin_fmaf(-0.5f, x2, 1.0f));
  const int m = k & 3;
  c = m == 0 ? cs : m == 1 ? -sn : m == 2 ? -cs : sn;
  s = m == 0 ? sn : m == 1 ? cs : m == 2 ? -sn : -cs;
}
// Fast-mode sampling without rejection loops (a wavefront would run a
// rejection loop until its unluckiest lane succeeds): the same
// distributions as unit_vector(random_in_unit_sphere()),
// random_in_unit_sphere() and random_in_unit_disk() (vec3.h:103-130);
// DESIGN.md §3.2.
__device__ __forceinline__ V3<float> unit_dir(Xoro &g) {
  float u, v, c, s;
  g.pair(u, v);
  const float z = __builtin_fmaf(-2.0f, u, 1.0f);
  const float r = dsqrt(__builtin_fmaf(-z, z, 1.0f));
  sincos2pi(v, c, s);
  return mk(r * c, r * s, z);
}
__device__ __forceinline__ V3<float> in_sphere_direct(Xoro &g) {
  const V3<float> d = unit_dir(g);
  float a, b;
  g.pair(a, b);
  const float c = g.uni();  // = the first of a pair, one step
  const float r = __builtin_fmaxf(a, __builtin_fmaxf(b, c));
  return mk(r * d.x, r * d.y, r * d.z);
}
__device__ __forceinline__ V3<float> in_disk_direct(Xoro &g) {
  float u, v, c, s;
  g.pair(u, v);
  const float r = dsqrt(u);
  sincos2pi(v, c, s);
  return mk(r * c, r * s, 0.0f);
}

// Replays a supplied glibc rand() stream: random_double() = rand()/(RAND_MAX+1.0)
struct StreamRng {
  const int32_t *p;
  int64_t pos, end;
  bool overflow;
  __device__ __forceinline__ double uni() {
    if (pos < end) return double(p[pos++]) / 2147483648.0;
    overflow = true;
    return 0.5;
  }
};

// random_double(-1,1) rtweekend.h:26-29: min + (max-min)*rd()
template <class R, class G> __device__ __forceinline__ R rd_m11(G &g) { return R(-1) + R(2) * R(g.uni()); }
// random_in_unit_sphere vec3.h:103-110: vec3::random(-1,1) draws z, y, x (GCC)
template <bool F, class R, class G> __device__ __forceinline__ V3<R> in_sphere(G &g) {
  for (;;) {
    const R z = rd_m11<R>(g);
    const R y = rd_m11<R>(g);
    const R x = rd_m11<R>(g);
    const V3<R> p = mk(x, y, z);
    if (dot<F>(p, p) >= R(1)) continue;
    return p;
  }
}
// random_in_unit_disk vec3.h:123-130: draws y, x (GCC)
template <bool F, class R, class G> __device__ __forceinline__ V3<R> in_disk(G &g) {
  for (;;) {
    const R y = rd_m11<R>(g);
    const R x = rd_m11<R>(g);
    if (madd<F>(y, y, x * x) >= R(1)) continue;
    return mk(x, y, R(0));
  }
}

// ---------------------------------------------------------------------------
// scene / camera views
// ---------------------------------------------------------------------------
template <class R> struct V4T;
template <> struct V4T<float> { using type = float4; };
template <> struct V4T<double> { using type = double4; };

// geom[k]  = {cx, cy, cz, |c|^2 - r^2} (float path) / {cx, cy, cz, r*r} (double path)
// shade0[k] = {1/r, albedo r, g, b}
// shade1[k] = {kind, fuzz (clamped), ir, 1/ir}
template <class R> struct SceneView {
  const typename V4T<R>::type *__restrict__ geom;
  const typename V4T<R>::type *__restrict__ sh0;
  const typename V4T<R>::type *__restrict__ sh1;
  int32_t n;
};

template <class R> struct Cam {
  V3<R> origin, llc, hor, ver, u, v;
  R lens;
};

// camera::get_ray camera.h:56-62
template <bool F, class R, class G>
__device__ __forceinline__ void get_ray(const Cam<R> &c, R s, R t, G &g, V3<R> &o, V3<R> &d) {
  V3<R> p;
  if constexpr (std::is_same<G, Xoro>::value) p = in_disk_direct(g);
  else p = in_disk<F, R>(g);
  const R rdx = c.lens * p.x, rdy = c.lens * p.y;
  const V3<R> off = mk(madd<F>(rdy, c.v.x, rdx * c.u.x), madd<F>(rdy, c.v.y, rdx * c.u.y),
                       madd<F>(rdy, c.v.z, rdx * c.u.z));
  o = mk(c.origin.x + off.x, c.origin.y + off.y, c.origin.z + off.z);
  d = mk((madd<F>(t, c.ver.x, madd<F>(s, c.hor.x, c.llc.x)) - c.origin.x) - off.x,
         (madd<F>(t, c.ver.y, madd<F>(s, c.hor.y, c.llc.y)) - c.origin.y) - off.y,
         (madd<F>(t, c.ver.z, madd<F>(s, c.hor.z, c.llc.z)) - c.origin.z) - off.z);
}

// hittable_list::hit over sphere::hit: closest root in the closed interval
// [t_min, closest_so_far]; ties go to the later object (sphere.h:36-41).
// The (hb >= 0 && cc >= 0) skip never changes the result: both roots are
// <= 0 < t_min there.  In the fast path the wave runs this
// loop in lockstep with sphere k in SGPRs.
template <bool F, class R>
__device__ __forceinline__ int32_t hit_world(const SceneView<R> &sc, V3<R> o, V3<R> d, R &t_hit) {
  const R a = dot<F>(d, d);
  const R inv_a = drcp(a);
  const R t_min = R(0.001);
  R t_max = R(INFINITY);
  int32_t best = -1;
#pragma unroll 4
  for (int32_t k = 0; k < sc.n; ++k) {
    const auto s = sc.geom[k];
    const R ocx = o.x - s.x, ocy = o.y - s.y, ocz = o.z - s.z;
    const R hb = madd<F>(ocz, d.z, madd<F>(ocy, d.y, ocx * d.x));
    const R cc = madd<F>(ocz, ocz, madd<F>(ocy, ocy, ocx * ocx)) - s.w;
    const R disc = madd<F>(hb, hb, -(a * cc));
    if (!(disc < R(0)) && !(hb >= R(0) && cc >= R(0))) {
      const R sq = dsqrt(disc);
      R root = F ? (-hb - sq) * inv_a : (-hb - sq) / a;
      bool ok = !(root < t_min || t_max < root);
      if (!ok) {
        root = F ? (-hb + sq) * inv_a : (-hb + sq) / a;
        ok = !(root < t_min || t_max < root);
      }
      if (ok) {
        t_max = root;
        best = k;
      }
    }
  }
  t_hit = t_max;
  return best;
}

// Packed form (the production loop).  On gfx950 a VALU op that reads an
// SGPR issues at HALF rate (4.07 vs 2.15 cycles per wave64 instruction,
// tools/valubench2.hip), while v_pk_fma_f32 — two FMAs per lane — issues at
// 4.1 cycles with or without an SGPR-pair operand.  So spheres are processed
// in PAIRS: pair q holds {cx, cy, cz, S} of spheres 2q and 2q+1 as float2s
// (SoA within the pair, 32 B), the ray terms are broadcast to both halves,
// and each of the 8 FMA-class ops per sphere becomes half of one
// v_pk_fma_f32.  Each half is an IEEE fma, so results are bit-identical to
// the scalar loop hit_world (and to the oracle).  Scenes are padded to a multiple of
// 2*GP spheres with a dummy {0, 0, 0, 1e30} that can never be a candidate.
typedef float f2v __attribute__((ext_vector_type(2)));
struct SpherePair {
  f2v cx, cy, cz, S;
};
constexpr float kDummyS = 1e30f;

template <int GP>
__device__ __forceinline__ int32_t hit_world_packed(const SpherePair *__restrict__ pairs, int32_t npairs, V3<float> o,
                                                    V3<float> d, float &t_hit
#if RTMI_STATS
                                                    , unsigned *stats
#endif
                                                    ) {
  const float a = dot<true>(d, d);
  const float inv_a = drcp(a);
  const float K = dot<true>(o, d);
  const float aL = a * dot<true>(o, o);
  const float n2a = -2.0f * a;
  const f2v DX = {d.x, d.x}, DY = {d.y, d.y}, DZ = {d.z, d.z}, KK = {K, K};
  const f2v MX = {n2a * o.x, n2a * o.x}, MY = {n2a * o.y, n2a * o.y}, MZ = {n2a * o.z, n2a * o.z};
  const f2v AA = {a, a}, AL = {aL, aL};
  const float t_min = 0.001f;
  float t_max = INFINITY;
  int32_t best = -1;
  auto resolve = [&](int32_t idx, float hb, float disc) {
#if RTMI_STATS
    stats[2] += 1;
#endif
    const float sq = dsqrt(disc);
    float root = (-hb - sq) * inv_a;
    bool ok = !(root < t_min || t_max < root);
    if (!ok) {
      root = (-hb + sq) * inv_a;
      ok = !(root < t_min || t_max < root);
    }
    if (ok) {
      t_max = root;
      best = idx;
    }
  };
  for (int32_t q = 0; q < npairs; q += GP) {
    SpherePair p[GP];
#pragma unroll
    for (int g = 0; g < GP; ++g) p[g] = pairs[q + g];
    f2v hb[GP], disc[GP];
    int ci[2 * GP];
    int any = 0;
#pragma unroll
    for (int g = 0; g < GP; ++g) {
      const f2v hz = __builtin_elementwise_fma(-p[g].cz, DZ, KK);
      hb[g] = __builtin_elementwise_fma(-p[g].cx, DX, __builtin_elementwise_fma(-p[g].cy, DY, hz));
      const f2v acc = __builtin_elementwise_fma(MX, p[g].cx, __builtin_elementwise_fma(MY, p[g].cy,
                      __builtin_elementwise_fma(MZ, p[g].cz, __builtin_elementwise_fma(AA, p[g].S, AL))));
      disc[g] = __builtin_elementwise_fma(hb[g], hb[g], -acc);
      // candidate iff disc >= +0 (sign clear): the full test resolves the rest
      ci[2 * g] = ~__float_as_int(disc[g].x);
      ci[2 * g + 1] = ~__float_as_int(disc[g].y);
      any |= ci[2 * g] | ci[2 * g + 1];
    }
#if RTMI_STATS
    stats[0] += 1;
    if (__ballot(any < 0)) stats[1] += 1;
    for (int k = 0; k < 2 * GP; ++k)
      if (__ballot(ci[k] < 0)) stats[3] += 1;
#endif
    if (any < 0) {
#pragma unroll
      for (int g = 0; g < GP; ++g) {
        if (ci[2 * g] < 0) resolve(2 * (q + g), hb[g].x, disc[g].x);
        if (ci[2 * g + 1] < 0) resolve(2 * (q + g) + 1, hb[g].y, disc[g].y);
      }
    }
  }
  t_hit = t_max;
  return best;
}

// ---------------------------------------------------------------------------
// BVH over the small spheres
// ---------------------------------------------------------------------------
// Same hit as hit_world_packed, bit for bit: the same expanded per-sphere
// arithmetic and root logic, and the reference's "later object wins ties"
// rule made order-independent (a root equal to the current t_max replaces
// the hit only for a larger sphere index), so the closest hit does not
// depend on the visiting order.  Boxes are conservative (inflated far beyond
// float error, rtmi_device.hip build_bvh), so a culled sphere is one the
// brute-force loop would have rejected.  Large spheres (the R=1000 ground,
// which bounds everything) stay in a brute-force packed list ("big").
// One node = 16 bytes = one ds_read_b128: per axis the box's lo and hi as
// IEEE halves in one dword (lo in bits 0-15), rounded OUTWARD from the
// double bounds (a half box contains the float box it replaces, so culling
// stays conservative; the slab test converts them for free with
// v_fma_mix_f32), and a link: >= 0 for an inner node = the skip index (next
// node when the box is missed; the first child is index + 1), < 0 for a
// leaf = ~(first << 4 | count) (the next node is index + 1 either way).
struct BvhNode {
  uint32_t x, y, z;
  int32_t link;
};
static_assert(sizeof(BvhNode) == 16, "BVH node is one 16-byte LDS read");
#ifndef RTMI_BVH_LEAF
#define RTMI_BVH_LEAF 4
#endif
constexpr int kLeafMax = RTMI_BVH_LEAF;
#ifndef RTMI_BIG_FACTOR
#define RTMI_BIG_FACTOR 4
#endif
#ifndef RTMI_BIG_GROUP
#define RTMI_BIG_GROUP 2
#endif
constexpr int kBigGroup = RTMI_BIG_GROUP;  // sphere pairs per step of the big-sphere loop
static_assert(kLeafMax >= 1 && kLeafMax <= 15, "leaf size");

// Uniform grid over the small spheres (RT_ACCEL_GRID): cells
// of size h over the box g0 + [0, n*h) of the spheres' margin-grown boxes.
// Cell c lists refs[cells[c] .. cells[c+1]): every sphere whose grown box
// overlaps it, as 16 x its scene index.  In LDS (stage_grid) each reference
// becomes a copy of its sphere's record, so the walk reads a sphere with one
// ds_read_b128 at the reference itself (grid_lds_bytes).
struct GridDesc {
  float g0[3], h[3], inv_h[3], g1[3];  // origin, cell size, 1/h, far corner
  int32_t n[3];
  int32_t ncells, nrefs;
  const uint32_t *cells;  // ncells + 1 first-reference indices
  const uint32_t *refs;
  uint32_t cells_off, idx_off;  // in LDS: the cell starts and the slot indices, bytes past the slots
};

struct Accel {
  const SpherePair *big;     // packed pairs of the big spheres (padded like the scene)
  const int32_t *big_idx;    // scene index of each big sphere slot (2 per pair)
  int32_t nbig_pairs;
  int32_t nnodes;
  const BvhNode *nodes;
  const float4 *sph;         // BVH: spheres in leaf order; grid: every sphere by scene index
  const int32_t *sph_idx;    // BVH: the leaf spheres' scene indices
  int32_t nsph;              // float4s of sph
  GridDesc grid;             // RT_ACCEL_GRID only
  int32_t bvh_global;        // BVH too large for LDS: walked in global memory (L2)
  // a grid over the LDS budget: the image stage_grid builds in LDS (slots,
  // cell starts, indices; offsets from 0) in global memory
  const char *grid_gmem;
};

// big_idx through the constant address space: wave-uniform scalar loads
__device__ __forceinline__ int32_t big_index(const Accel &a, int slot) {
  typedef const __attribute__((address_space(4))) int32_t *cidx_t;
  return ((cidx_t)(size_t)a.big_idx)[slot];
}

// The BVH lives in LDS during a launch (dynamic shared memory, staged by
// every block at its start): the traversal is a chain of dependent node
// loads, ~100 cycles from LDS against ~500+ from L2.  Layout: nnodes 16-byte
// nodes, then nsph sphere float4s, then nsph uint16 scene indices (the BVH is
// only offered for scenes of < 65536 spheres).
extern __shared__ float4 rtmi_bvh_lds[];
__host__ __device__ constexpr size_t bvh_lds_bytes(int32_t nnodes, int32_t nsph) {
  return size_t(nnodes + nsph) * 16 + size_t(nsph) * 2;
}

__device__ __forceinline__ void stage_bvh(const Accel &g) {
  if (!g.bvh_global) {  // (a BVH over the LDS budget stays in global memory)
    const float4 *nodes = reinterpret_cast<const float4 *>(g.nodes);
    for (int i = threadIdx.x; i < g.nnodes; i += blockDim.x) rtmi_bvh_lds[i] = nodes[i];
    for (int i = threadIdx.x; i < g.nsph; i += blockDim.x) rtmi_bvh_lds[g.nnodes + i] = g.sph[i];
    uint16_t *idx = reinterpret_cast<uint16_t *>(rtmi_bvh_lds + g.nnodes + g.nsph);
    for (int i = threadIdx.x; i < g.nsph; i += blockDim.x) idx[i] = uint16_t(g.sph_idx[i]);
  }
  __syncthreads();
}

// LDS addresses as 32-bit integers (the offset of a shared variable within
// the workgroup's LDS) and a float4 read at one: a ds_read_b128 at the value
// itself.  (Device pass only; the host pass never runs these.)
__device__ __forceinline__ uint32_t lds_address(const void *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return uint32_t(size_t((const __attribute__((address_space(3))) char *)p));
#else
  return uint32_t(size_t(p));
#endif
}
__device__ __forceinline__ float4 lds_sphere(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __attribute__((address_space(3))) float4 *p = (const __attribute__((address_space(3))) float4 *)(size_t)addr;
  return make_float4(p->x, p->y, p->z, p->w);
#else
  return make_float4(0.f, 0.f, 0.f, float(addr));
#endif
}

// Grid LDS layout ("record slots"): one 16-byte sphere record {c, S} per slot
// — first the big spheres' slots (2 x nbig_pairs, dummies included), then
// every cell's references in cell order, each a copy of the record of the
// sphere it lists — then ncells + 1 uint32 cell starts (the LDS addresses of
// their first slots), then one uint16 scene index per slot.  The walk reads a
// sphere with one ds_read_b128 at the slot (no reference indirection), and
// names a hit by its slot's LDS address (a "key"); the scene index is read
// from the index table only for an exact tie and once at the walk's end.
__host__ __device__ constexpr size_t grid_lds_bytes(int32_t nbig_slots, int32_t ncells, int32_t nrefs) {
  return size_t(nbig_slots + nrefs) * 16 + (size_t(ncells) + 1) * 4 + (size_t(nbig_slots + nrefs) * 2 + 3) / 4 * 4;
}

// The grid descriptor in LDS (staged with the grid): the walk setup reads its
// fields there instead of holding them in scalar registers, which overflowed
// the kernel's SGPR budget into VGPR lanes read back with v_readlane (15 per
// loop pass, 3 now; config 2 -0.6 to -0.8%, profiles/r04/ab_variants*.txt).
__shared__ GridDesc rtmi_grid_desc;
__device__ __forceinline__ void stage_grid(const Accel &g) {
  const int32_t nbs = 2 * g.nbig_pairs, nrec = nbs + g.grid.nrefs;
  float4 *rec = rtmi_bvh_lds;
  uint32_t *c = reinterpret_cast<uint32_t *>(rec + nrec);
  uint16_t *ix = reinterpret_cast<uint16_t *>(c + g.grid.ncells + 1);
  const uint32_t rec_base = lds_address(rec);
  if (threadIdx.x == 0) rtmi_grid_desc = g.grid;
  for (int i = threadIdx.x; i < nrec; i += blockDim.x) {
    const int32_t k = i < nbs ? g.big_idx[i] : int32_t(g.grid.refs[i - nbs] >> 4);  // dummies: -1
    rec[i] = k < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : g.sph[k];
    ix[i] = uint16_t(k < 0 ? 0 : k);
  }
  for (int i = threadIdx.x; i <= g.grid.ncells; i += blockDim.x)
    c[i] = rec_base + 16u * (uint32_t(nbs) + g.grid.cells[i]);
  __syncthreads();
}
// A grid walked in global memory (Accel::grid_gmem): only the descriptor is
// staged; slots, cell starts and indices are read at gmem + the same offsets.
__device__ __forceinline__ void stage_grid_desc(const Accel &g) {
  if (threadIdx.x == 0) rtmi_grid_desc = g.grid;
  __syncthreads();
}
// a uint32 at an LDS address
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(3))) uint32_t *)(size_t)addr;
#else
  return addr;
#endif
}
// a uint16 at an LDS address
__device__ __forceinline__ uint32_t lds_u16(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(3))) uint16_t *)(size_t)addr;
#else
  return addr;
#endif
}

// Inverse direction for culling only (slab tests, grid cell faces): |d_i|
// clamped to >= 1e-20 (see hit_world_bvh), then the hardware reciprocal
// (v_rcp_f32, ~1 ulp) instead of a correctly rounded division: the
// structures' margins are ~1e4 times larger than that error, and no hit
// result depends on it (the sphere tests use the exact inv_a).
__device__ __forceinline__ float safe_inv(float v) {
  const float c = __builtin_fabsf(v) < 1e-20f ? __builtin_copysignf(1e-20f, v) : v;
  return __builtin_amdgcn_rcpf(c);
}

#ifndef RTMI_TRACE_PHASES
#define RTMI_TRACE_PHASES 0
#endif


#if RTMI_TRACE_PHASES
// analysis only: wave-level cycles (s_memtime) of the grid walk's phases:
// [0] big spheres, [1] clip + DDA setup, [2] cell walk
struct PhaseClock { unsigned long long c[3]; };
#endif

// Per-segment ray terms of the expanded sphere test, shared
// by the accelerated walks.  Plain scalars, not a struct: a struct here ends
// up in scratch memory (its fields get combined into vector loads before
// they can be promoted to registers).
#define RTMI_RAY_TERMS(o, d)                                    \
  const float a = dot<true>(d, d);                              \
  const float inv_a = drcp(a);                                  \
  const float K = dot<true>(o, d);                              \
  const float aL = a * dot<true>(o, o);                         \
  const float n2a = -2.0f * a;                                  \
  const float mx = n2a * o.x, my = n2a * o.y, mz = n2a * o.z;

// sphere {c, S = |c|^2 - r^2}: hb = (o-c).d, disc = hb^2 - a(|o-c|^2 - r^2)
__device__ __forceinline__ void sphere_test(const float4 sp, V3<float> d, float K, float a, float aL, float mx,
                                            float my, float mz, float &hb, float &disc) {
  hb = __builtin_fmaf(-sp.x, d.x, __builtin_fmaf(-sp.y, d.y, __builtin_fmaf(-sp.z, d.z, K)));
  const float ac = __builtin_fmaf(mx, sp.x, __builtin_fmaf(my, sp.y, __builtin_fmaf(mz, sp.z, __builtin_fmaf(a, sp.w, aL))));
  disc = __builtin_fmaf(hb, hb, -ac);
}

// sphere.h:30-38 root logic, closed interval [0.001, t_max]; the reference's
// "later object wins ties" (hittable_list.h:25-31) made order-independent: a
// root equal to t_max replaces the hit only for a larger scene index, so any
// visiting order gives the in-order loop's hit.  The second root counts only
// when the first is rejected; both are formed and selected (no branch:
// measured faster than forming the second only when needed).
__device__ __forceinline__ void resolve_root(int32_t idx, float hb, float disc, float inv_a, float &t_max,
                                             int32_t &best) {
  const float sq = dsqrt(disc);
  const float r1 = (-hb - sq) * inv_a, r2 = (-hb + sq) * inv_a;
  const bool later = idx > best;
  // bitwise, not short-circuit: compare masks combined by scalar ops instead
  // of nested exec-mask branches (config 2: 23.55 -> 23.25 ms,
  // profiles/r03/ab_accept.txt)
  const bool ok1 = !(r1 < 0.001f) & ((r1 < t_max) | ((r1 == t_max) & later));
  const bool ok2 = !(r2 < 0.001f) & ((r2 < t_max) | ((r2 == t_max) & later));
  if (ok1 || ok2) {
    t_max = ok1 ? r1 : r2;
    best = idx;
  }
}

// resolve_root for the grid walk, whose hits are named by record-slot keys
// (stage_grid): the same acceptance, with the scene indices read from the
// slot index table only for an exact tie (r == t_max), which is rare, instead
// of carried per candidate.  best_key -1: no hit yet.
template <bool GMEM = false>
__device__ __forceinline__ void resolve_key(uint32_t key, float hb, float disc, float inv_a, float &t_max,
                                            int32_t &best_key, uint32_t idx_base, const char *gmem = nullptr) {
  const float sq = dsqrt(disc);
  const float r1 = (-hb - sq) * inv_a, r2 = (-hb + sq) * inv_a;
  const bool g1 = !(r1 < 0.001f), g2 = !(r2 < 0.001f);
  bool ok1 = g1 & (r1 < t_max), ok2 = g2 & (r2 < t_max);
  const bool e1 = g1 & (r1 == t_max), e2 = g2 & (r2 == t_max);
  if (__builtin_expect(e1 | e2, 0)) {
    const uint32_t rec_base = GMEM ? 0u : lds_address(rtmi_bvh_lds);
    const uint32_t bk = best_key < 0 ? key : uint32_t(best_key);
    auto u16 = [&](uint32_t a) {
      if constexpr (GMEM) return uint32_t(*reinterpret_cast<const uint16_t *>(gmem + a));
      else return lds_u16(a);
    };
    const bool later = (best_key < 0) | (u16(idx_base + ((key - rec_base) >> 3)) >
                                         u16(idx_base + ((bk - rec_base) >> 3)));
    ok1 |= e1 & later;
    ok2 |= e2 & later;
  }
  if (ok1 || ok2) {
    t_max = ok1 ? r1 : r2;
    best_key = int32_t(key);
  }
}

// The big spheres (the ones kept out of the BVH / grid: the R = 1000 ground
// and the r = 1 spheres) by the packed brute-force loop: group data and scene
// indices through scalar loads, each half of a v_pk_fma_f32 an IEEE fma.
// KEYS (the grid walk): best is a record-slot key, slot j's key rec_base + 16 j.
template <int GP, bool KEYS = false, bool GMEM = false>
__device__ __forceinline__ void hit_big(const Accel &acc_s, V3<float> d, float K, float a, float aL, float mx, float my,
                                        float mz, float inv_a, float &t_max, int32_t &best
#if RTMI_STATS
                                        , unsigned *stats
#endif
                                        ) {
  static_assert(GP == 2, "the big-sphere loop resolves groups of two pairs");
  const f2v DX = {d.x, d.x}, DY = {d.y, d.y}, DZ = {d.z, d.z}, KK = {K, K};
  const f2v MX = {mx, mx}, MY = {my, my}, MZ = {mz, mz};
  const f2v AA = {a, a}, AL = {aL, aL};
  typedef const __attribute__((address_space(4))) SpherePair *cpair_t;
  const cpair_t cp = (cpair_t)(size_t)acc_s.big;
  auto pair = [&](int q, f2v &hb, f2v &disc) {
    const f2v cx = cp[q].cx, cy = cp[q].cy, cz = cp[q].cz, S = cp[q].S;
    const f2v hz = __builtin_elementwise_fma(-cz, DZ, KK);
    hb = __builtin_elementwise_fma(-cx, DX, __builtin_elementwise_fma(-cy, DY, hz));
    const f2v ac = __builtin_elementwise_fma(MX, cx, __builtin_elementwise_fma(MY, cy,
                   __builtin_elementwise_fma(MZ, cz, __builtin_elementwise_fma(AA, S, AL))));
    disc = __builtin_elementwise_fma(hb, hb, -ac);
  };
  // candidate iff disc >= +0 (sign clear; the dummies never are)
  auto cand = [](float x, int bit) { return (__float_as_int(x) >= 0 ? 1u : 0u) << bit; };
  for (int32_t q = 0; q < acc_s.nbig_pairs; q += 2) {
    f2v hb0, d0, hb1, d1;
    pair(q, hb0, d0);
    pair(q + 1, hb1, d1);
    // one wave-uniform branch per group when no lane has a candidate, then
    // per slot (measured: resolving one candidate per lane per round, with
    // the slot picked by selects, is slower)
    const unsigned m = cand(d0.x, 0) | cand(d0.y, 1) | cand(d1.x, 2) | cand(d1.y, 3);
    if (m) {
#if RTMI_STATS
      if (__lane_id() == __builtin_ctzll(__ballot(1))) stats[4] += 1;
#endif
      auto res = [&](int slot, float hb, float disc) {
        if constexpr (KEYS)  // the big slots' keys are in scene order: the plain tie rule
          resolve_root(int32_t((GMEM ? 0u : lds_address(rtmi_bvh_lds)) + 16u * uint32_t(slot)), hb, disc, inv_a, t_max,
                       best);
        else
          resolve_root(big_index(acc_s, slot), hb, disc, inv_a, t_max, best);
      };
      if (m & 1u) res(2 * q, hb0.x, d0.x);
      if (m & 2u) res(2 * q + 1, hb0.y, d0.y);
      if (m & 4u) res(2 * q + 2, hb1.x, d1.x);
      if (m & 8u) res(2 * q + 3, hb1.y, d1.y);
    }
  }
}

// Closest hit through the uniform grid (RT_ACCEL_GRID, staged in LDS by
// stage_grid): the big spheres brute force, then a 3D-DDA walk over the
// cells the ray crosses inside [entry, t_max], testing each cell's spheres
// (one LDS read for the cell's reference range, then per sphere its scene
// index and its record) with exactly the brute-force arithmetic and the
// order-independent tie rule.  (Measured and not kept: cells padded to
// records of four references tested unrolled — more VALU work per cell.)  The walk stops at the first cell whose exit
// lies at or beyond the closest hit so far.  Exact: every
// sphere is listed in every cell its grown box overlaps, the grow margin
// (>= 1e-3 of the sphere's scale) is orders of magnitude above the float
// error of the cell boundaries (each computed directly from the cell index,
// never accumulated), so the cell the DDA holds for any accepted hit point
// lists that sphere; a sphere tested in several cells gives the same root
// each time.  FLAT_Y: the grid has one cell layer in y (the final scene's
// 20 x 1 x 20) — the same walk with the y axis' stepping state dropped: a y
// face only ends the walk (5 VGPRs fewer in the loop).
template <int GP, bool FLAT_Y = false, bool GMEM = false>
__device__ __forceinline__ int32_t hit_world_grid(const Accel &acc_s, V3<float> o, V3<float> d, float &t_hit,
                                                  uint32_t &hit_key
#if RTMI_STATS
                                                  , unsigned *gstats
#endif
#if RTMI_TRACE_PHASES
                                                  , PhaseClock &pc
#endif
                                                  ) {
#if RTMI_TRACE_PHASES
  const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
  RTMI_RAY_TERMS(o, d)
  // the record slots (grid_lds_bytes); the slot index table's address from
  // the kernel arguments, a scalar (from the LDS descriptor it would be a
  // VGPR held through the walk, which the kernel has none to spare of)
  // (GMEM: the same layout in global memory at acc_s.grid_gmem, offsets from 0)
  const char *const gm = GMEM ? acc_s.grid_gmem : nullptr;
  const uint32_t base = GMEM ? 0u : lds_address(rtmi_bvh_lds), idx_base = base + acc_s.grid.idx_off;
  auto rd_u32 = [&](uint32_t addr) {
    if constexpr (GMEM) return *reinterpret_cast<const uint32_t *>(gm + addr);
    else return lds_u32(addr);
  };
  auto rd_u16 = [&](uint32_t addr) {
    if constexpr (GMEM) return uint32_t(*reinterpret_cast<const uint16_t *>(gm + addr));
    else return lds_u16(addr);
  };
  auto rd_sphere = [&](uint32_t addr) {
    if constexpr (GMEM) return *reinterpret_cast<const float4 *>(gm + addr);
    else return lds_sphere(addr);
  };
  float t_max = INFINITY;
  int32_t best_a = -1;  // the hit's record-slot key; -1: no hit yet
  hit_big<GP, true, GMEM>(acc_s, d, K, a, aL, mx, my, mz, inv_a, t_max, best_a
#if RTMI_STATS
              , gstats
#endif
              );
#if RTMI_TRACE_PHASES
  const unsigned long long tp1 = __builtin_amdgcn_s_memtime();
  pc.c[0] += tp1 - tp0;
  unsigned long long tp2 = tp1;
#endif
  const GridDesc &G = rtmi_grid_desc;  // (stage_grid)
  const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
  const float ox = -o.x * ix, oy = -o.y * iy, oz = -o.z * iz;
  // the grid box, clipped to [0, t_max]
  const float bx0 = __builtin_fmaf(G.g0[0], ix, ox), bx1 = __builtin_fmaf(G.g1[0], ix, ox);
  const float by0 = __builtin_fmaf(G.g0[1], iy, oy), by1 = __builtin_fmaf(G.g1[1], iy, oy);
  const float bz0 = __builtin_fmaf(G.g0[2], iz, oz), bz1 = __builtin_fmaf(G.g1[2], iz, oz);
  const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(bx0, bx1), __builtin_fminf(by0, by1)),
                                      __builtin_fmaxf(__builtin_fminf(bz0, bz1), 0.0f));
  const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(bx0, bx1), __builtin_fmaxf(by0, by1)),
                                     __builtin_fminf(__builtin_fmaxf(bz0, bz1), t_max));
  if (tnear <= tfar) {
    const uint32_t cells = base + G.cells_off;
    // entry cell: the cell of o + tnear*d, clamped into the grid
    auto cell_of = [&](float p, int ax) {
      const int c = int(__builtin_floorf((p - G.g0[ax]) * G.inv_h[ax]));
      return c < 0 ? 0 : (c >= G.n[ax] ? G.n[ax] - 1 : c);
    };
    const int cx = cell_of(__builtin_fmaf(tnear, d.x, o.x), 0);
    const int cy = FLAT_Y ? 0 : cell_of(__builtin_fmaf(tnear, d.y, o.y), 1);
    const int cz = cell_of(__builtin_fmaf(tnear, d.z, o.z), 2);
    // Per axis: after k steps on it the current cell's far face lies at
    // t = fma(k, dt, t0) (t0 the entry cell's far face, dt = h/|d_axis|), and
    // the walk leaves the grid when it would step past kmax.  (Only which
    // cells are visited depends on these roundings, never a hit: DESIGN.md
    // §4.5's argument needs face parameters within ~1e-6 of the truth, the
    // margins being >= 1e-3.)
    float t0x, t0y, t0z, dtx, dty, dtz, kmx, kmy, kmz;
    // The step direction comes from the culling inverse, not from d: safe_inv
    // gives -0.0 the inverse -1e20, so `d >= 0` (true for -0.0) would pick the
    // far face on the wrong side and step into cells the ray never enters.
    auto axis = [&](float inv, float oo, int c, int ax, float &t0, float &dt, float &kmax) {
      const bool pos = inv >= 0.0f;
      t0 = __builtin_fmaf(__builtin_fmaf(float(c + (pos ? 1 : 0)), G.h[ax], G.g0[ax]), inv, oo);
      dt = __builtin_fabsf(G.h[ax] * inv);
      kmax = float(pos ? G.n[ax] - 1 - c : c);
    };
    axis(ix, ox, cx, 0, t0x, dtx, kmx);
    if constexpr (FLAT_Y) {  // the one layer's far y face (axis() at c = 0, no steps)
      t0y = __builtin_fmaf(__builtin_fmaf(iy >= 0.0f ? 1.0f : 0.0f, G.h[1], G.g0[1]), iy, oy);
      dty = kmy = 0.0f;
    } else {
      axis(iy, oy, cy, 1, t0y, dty, kmy);
    }
    axis(iz, oz, cz, 2, t0z, dtz, kmz);
    float kx = 0.0f, ky = 0.0f, kz = 0.0f, tnx = t0x, tny = t0y, tnz = t0z;
    // the LDS address of the current cell's start, stepped by 4 x the cell step
    uint32_t cell = cells + 4u * uint32_t(cx + G.n[0] * (cy + G.n[1] * cz));
    const int dcx = ix >= 0.0f ? 4 : -4, dcy = iy >= 0.0f ? 4 * G.n[0] : -4 * G.n[0];
    const int dcz = iz >= 0.0f ? 4 * G.n[0] * G.n[1] : -4 * G.n[0] * G.n[1];
#if RTMI_TRACE_PHASES
    tp2 = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
#if RTMI_STATS
      gstats[0] += 1;
      if (__lane_id() == __builtin_ctzll(__ballot(1))) gstats[2] += 1;
#endif
      const uint32_t re = rd_u32(cell + 4u);  // (with the next one: a ds_read2_b32)
      // Deferred root resolution: a lane keeps its first candidate of the
      // cell and resolves it after the cell's sphere loop (a second candidate
      // resolves the kept one first).  A wave then runs the resolution about
      // once per cell instead of at every sphere where some lane has a
      // candidate (tools/grid_sim.c: 3.4 instead of 4.8 per wave-segment).
      // The result is the same: resolve_root's acceptance is order-independent
      // (the closest root, ties to the larger index), and the walk's exit
      // test comes after the cell's resolutions either way.  (kNoKey: none —
      // an explicit sentinel no LDS address can take, not 0, which slot 0
      // would be if nothing preceded the dynamic LDS)
      constexpr uint32_t kNoKey = 0xFFFFFFFFu;
      uint32_t kaddr = kNoKey;
      float khb = 0.0f, kdisc = 0.0f;
      for (uint32_t r = rd_u32(cell); r < re; r += 16u) {
#if RTMI_STATS
        gstats[1] += 1;
        if (__lane_id() == __builtin_ctzll(__ballot(1))) gstats[3] += 1;
#endif
        float hb, disc;
        sphere_test(rd_sphere(r), d, K, a, aL, mx, my, mz, hb, disc);
        if (!(disc < 0.0f)) {
          if (kaddr != kNoKey) {
#if RTMI_STATS
            if (__lane_id() == __builtin_ctzll(__ballot(1))) gstats[4] += 1;
#endif
            resolve_key<GMEM>(kaddr, khb, kdisc, inv_a, t_max, best_a, idx_base, gm);
          }
          kaddr = r;
          khb = hb;
          kdisc = disc;
        }
      }
      if (kaddr != kNoKey) {
#if RTMI_STATS
        if (__lane_id() == __builtin_ctzll(__ballot(1))) gstats[4] += 1;
#endif
        resolve_key<GMEM>(kaddr, khb, kdisc, inv_a, t_max, best_a, idx_base, gm);
      }
      const float texit = __builtin_fminf(tnx, __builtin_fminf(tny, tnz));
      if constexpr (FLAT_Y) {
        // the same step without nested branches: x when its face is nearest
        // (ties to x), the y face ends the walk, else z (selects: 19.92 vs
        // 20.06 ms, profiles/r03/ab_dda_select_shade_uniform.txt)
        const bool sx = (tnx <= tny) & (tnx <= tnz);
        const bool sy = !sx & (tny <= tnz);
        const bool leave = !(texit < t_max) | sy | ((sx ? kx : kz) >= (sx ? kmx : kmz));
        if (leave) break;
        kx = sx ? kx + 1.0f : kx;
        kz = sx ? kz : kz + 1.0f;
        tnx = sx ? __builtin_fmaf(kx, dtx, t0x) : tnx;
        tnz = sx ? tnz : __builtin_fmaf(kz, dtz, t0z);
        cell += sx ? dcx : dcz;
        continue;
      }
      if (!(texit < t_max)) break;  // the closest hit so far lies in the cells walked
      if (tnx <= tny && tnx <= tnz) {
        if (kx >= kmx) break;  // leaves the grid
        kx += 1.0f;
        tnx = __builtin_fmaf(kx, dtx, t0x);
        cell += dcx;
      } else if (tny <= tnz) {
        if (FLAT_Y || ky >= kmy) break;  // leaves the grid
        ky += 1.0f;
        tny = __builtin_fmaf(ky, dty, t0y);
        cell += dcy;
      } else {
        if (kz >= kmz) break;
        kz += 1.0f;
        tnz = __builtin_fmaf(kz, dtz, t0z);
        cell += dcz;
      }
    }
  }
#if RTMI_TRACE_PHASES
  {
    const unsigned long long tp3 = __builtin_amdgcn_s_memtime();
    pc.c[1] += tp2 - tp1;
    pc.c[2] += tp3 - tp2;
  }
#endif
  t_hit = t_max;
  // the scene index of the hit slot (a miss reads slot 0's, unused)
  hit_key = best_a < 0 ? base : uint32_t(best_a);
  const int32_t k = int32_t(rd_u16(idx_base + ((hit_key - base) >> 3)));
  return best_a < 0 ? -1 : k;
}

template <int GP>
__device__ __forceinline__ int32_t hit_world_bvh(const Accel &acc_s, V3<float> o, V3<float> d, float &t_hit
#if RTMI_STATS
                                                 , unsigned *bstats
#endif
                                                 ) {
  RTMI_RAY_TERMS(o, d)
  float t_max = INFINITY;
  int32_t best = -1;
  // 1. big spheres: the packed brute-force loop
  hit_big<GP>(acc_s, d, K, a, aL, mx, my, mz, inv_a, t_max, best
#if RTMI_STATS
              , bstats
#endif
  );
  // 2. the BVH (staged in LDS by stage_bvh, or in global memory when it is
  // over the LDS budget: bvh_global, a wave-uniform choice), stackless:
  // per-lane walk of the DFS node array with skip links
  // inverse direction with |d_i| clamped to >= 1e-20: no infinities, so no
  // 0*inf or inf-inf NaNs in the slab test (min/max would not ignore them
  // reliably).  The clamp moves the ray by a negligible angle; a ray running
  // parallel to a slab plane within ~1e-6 of it cannot reach a sphere, which
  // sits at least the box margin inside every face.
  const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
  // slab distances as one fma per plane: (b - o) * i = fma(b, i, -o*i); the
  // box margin covers the different rounding
  const float ox = -o.x * ix, oy = -o.y * iy, oz = -o.z * iz;
  auto lo16 = [](uint32_t w) { return float(__builtin_bit_cast(_Float16, uint16_t(w))); };
  auto hi16 = [](uint32_t w) { return float(__builtin_bit_cast(_Float16, uint16_t(w >> 16))); };
  auto walk = [&](auto in_global) {
    constexpr bool GLOBAL = decltype(in_global)::value;
    const uint4 *nodes = GLOBAL ? reinterpret_cast<const uint4 *>(acc_s.nodes) : reinterpret_cast<const uint4 *>(rtmi_bvh_lds);
    const float4 *sph = GLOBAL ? acc_s.sph : rtmi_bvh_lds + acc_s.nnodes;
    const uint16_t *lds_idx = reinterpret_cast<const uint16_t *>(rtmi_bvh_lds + acc_s.nnodes + acc_s.nsph);
    int32_t node = 0;
    while (node < acc_s.nnodes) {
      const uint4 nd = nodes[node];
      const float tx0 = __builtin_fmaf(lo16(nd.x), ix, ox), tx1 = __builtin_fmaf(hi16(nd.x), ix, ox);
      const float ty0 = __builtin_fmaf(lo16(nd.y), iy, oy), ty1 = __builtin_fmaf(hi16(nd.y), iy, oy);
      const float tz0 = __builtin_fmaf(lo16(nd.z), iz, oz), tz1 = __builtin_fmaf(hi16(nd.z), iz, oz);
      // slab interval clipped to [0, t_max].  No slack is needed: a sphere
      // that can be hit lies >= the box margin inside the box, so its chord
      // starts after tnear and ends before tfar by far more than rounding, and
      // a hit at t_hit >= 0.001 with t_hit <= t_max (ties included) keeps the
      // box entered.  Half-precision bounds only make the box larger.
      const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx0, tx1), __builtin_fminf(ty0, ty1)),
                                          __builtin_fmaxf(__builtin_fminf(tz0, tz1), 0.0f));
      const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx0, tx1), __builtin_fmaxf(ty0, ty1)),
                                         __builtin_fminf(__builtin_fmaxf(tz0, tz1), t_max));
      const bool enter = tnear <= tfar;
      const int32_t link = int32_t(nd.w);
#if RTMI_STATS
      bstats[0] += 1;
      if (__lane_id() == __builtin_ctzll(__ballot(1))) bstats[2] += 1;
#endif
      if (enter && link < 0) {
        const int32_t first = (~link) >> 4, cnt = (~link) & 15;
#if RTMI_STATS
        bstats[1] += cnt;
#endif
        for (int32_t k = first; k < first + cnt; ++k) {
#if RTMI_STATS
          if (__lane_id() == __builtin_ctzll(__ballot(1))) bstats[3] += 1;
#endif
          float hb, disc;
          sphere_test(sph[k], d, K, a, aL, mx, my, mz, hb, disc);
          if (!(disc < 0.0f)) {
#if RTMI_STATS
            if (__lane_id() == __builtin_ctzll(__ballot(1))) bstats[4] += 1;
#endif
            resolve_root(GLOBAL ? acc_s.sph_idx[k] : int32_t(lds_idx[k]), hb, disc, inv_a, t_max, best);
          }
        }
      }
      node = (enter || link < 0) ? node + 1 : link;
    }
  };
  if (acc_s.bvh_global)
    walk(std::true_type{});
  else
    walk(std::false_type{});
  t_hit = t_max;
  return best;
}

// material::scatter material.h:15-97.  Returns true if the ray scattered.
template <bool F, class R, class G>
__device__ __forceinline__ bool scatter(const SceneView<R> &sc, int32_t k, V3<R> din, V3<R> normal,
                                        bool front, G &g, V3<R> &atten, V3<R> &dout) {
  const auto s0 = sc.sh0[k];
  const auto s1 = sc.sh1[k];
  const int kind = int(s1.x);
  if (kind == RT_MAT_LAMBERTIAN) {  // material.h:19-31
    V3<R> ru;
    if constexpr (std::is_same<G, Xoro>::value) ru = unit_dir(g);
    else ru = unit<F>(in_sphere<F, R>(g));
    V3<R> dir = mk(normal.x + ru.x, normal.y + ru.y, normal.z + ru.z);
    if (near_zero(dir)) dir = normal;
    dout = dir;
    atten = mk(s0.y, s0.z, s0.w);
    return true;
  }
  if (kind == RT_MAT_METAL) {  // material.h:40-49
    const V3<R> refl = reflect<F>(unit<F>(din), normal);
    V3<R> rv;
    if constexpr (std::is_same<G, Xoro>::value) rv = in_sphere_direct(g);
    else rv = in_sphere<F, R>(g);
    const R fz = s1.y;
    const V3<R> dir = mk(madd<F>(fz, rv.x, refl.x), madd<F>(fz, rv.y, refl.y), madd<F>(fz, rv.z, refl.z));
    dout = dir;
    atten = mk(s0.y, s0.z, s0.w);
    return dot<F>(dir, normal) > R(0);
  }
  // dielectric material.h:60-85
  atten = mk(R(1), R(1), R(1));
  const R ratio = front ? s1.w : s1.z;
  const V3<R> ud = unit<F>(din);
  const R cos_theta = dfmin(dot<F>(mk(-ud.x, -ud.y, -ud.z), normal), R(1));
  const R sin_theta = dsqrt(madd<F>(-cos_theta, cos_theta, R(1)));
  const bool cannot_refract = ratio * sin_theta > R(1);
  if (cannot_refract || reflectance<F>(cos_theta, ratio) > R(g.uni()))
    dout = reflect<F>(ud, normal);
  else
    dout = refract<F>(ud, normal, ratio, cos_theta);
  return true;
}

// The fast kernels' form of scatter<true, float, Xoro>: the same arithmetic
// and random draws per lane, arranged so that the parts materials share run
// once per wave instead of once per material branch (a wave's lanes hit all
// three materials at once):
//  * every material's first draw is one xoroshiro step: lambertian and metal
//    take its (u, v) pair for unit_dir, the dielectric its top 24 bits as
//    g.uni() — the same u;
//  * metal and dielectric share unit(din) and reflect(unit(din), n).
// The dielectric draws its uniform only when it can refract (the short
// circuit of material.h:80): a dielectric lane that cannot refract gets its
// generator state back.
// inv_len = 1/sqrt(din.din) (correctly rounded), as unit() computes it; the
// caller shares it with the sky of the wave's missed lanes.
// (s0, s1 = shade0[k], shade1[k]: the caller loads the hit sphere's records
// together, in one memory round trip)
__device__ __forceinline__ bool scatter_fast(const float4 s0, const float4 s1, V3<float> din, V3<float> normal,
                                             bool front, Xoro &g, V3<float> &atten, V3<float> &dout, float inv_len) {
  const int kind = int(s1.x);
  const Xoro g0 = g;
  float u, v;
  g.pair(u, v);  // the first draw of every material
  V3<float> ud = mk(0.f, 0.f, 0.f), refl = mk(0.f, 0.f, 0.f);
  if (kind != RT_MAT_LAMBERTIAN) {  // metal, dielectric: unit(din), reflect
    ud = scale(inv_len, din);
    refl = reflect<true>(ud, normal);
  }
  if (kind != RT_MAT_DIELECTRIC) {  // lambertian, metal: unit_dir from (u, v)
    const float z = __builtin_fmaf(-2.0f, u, 1.0f);
    const float r = dsqrt(__builtin_fmaf(-z, z, 1.0f));
    float c, sn;
    sincos2pi(v, c, sn);
    const V3<float> ru = mk(r * c, r * sn, z);
    atten = mk(s0.y, s0.z, s0.w);
    if (kind == RT_MAT_LAMBERTIAN) {  // material.h:19-31
      V3<float> dir = mk(normal.x + ru.x, normal.y + ru.y, normal.z + ru.z);
      if (near_zero(dir)) dir = normal;
      dout = dir;
      return true;
    }
    // metal material.h:40-49: a point in the ball = ru * max of three uniforms
    float a, b;
    g.pair(a, b);
    const float cc = g.uni();  // = the first of a pair, one step
    const float rr = __builtin_fmaxf(a, __builtin_fmaxf(b, cc));
    const V3<float> rv = mk(rr * ru.x, rr * ru.y, rr * ru.z);
    const float fz = s1.y;
    const V3<float> dir = mk(__builtin_fmaf(fz, rv.x, refl.x), __builtin_fmaf(fz, rv.y, refl.y),
                             __builtin_fmaf(fz, rv.z, refl.z));
    dout = dir;
    return dot<true>(dir, normal) > 0.0f;
  }
  // dielectric material.h:60-85
  atten = mk(1.f, 1.f, 1.f);
  const float ratio = front ? s1.w : s1.z;
  const float cos_theta = dfmin(dot<true>(mk(-ud.x, -ud.y, -ud.z), normal), 1.0f);
  const float sin_theta = dsqrt(__builtin_fmaf(-cos_theta, cos_theta, 1.0f));
  const bool cannot_refract = ratio * sin_theta > 1.0f;
  if (cannot_refract) g = g0;  // the uniform is not drawn
  // Schlick with r0 precomputed per face by the host (rt_ctx_set_scene):
  // reflectance<true>(cos_theta, ratio) without its division
  const float r0 = front ? s1.y : s0.y;
  if (cannot_refract || __builtin_fmaf(1.0f - r0, pow5(1.0f - cos_theta), r0) > u)
    dout = refl;
  else
    dout = refract<true>(ud, normal, ratio, cos_theta);
  return true;
}

// Hit record (sphere.h:43-53, hittable.h:23-26) for sphere k at t.
template <bool F, class R>
__device__ __forceinline__ void hit_record(const SceneView<R> &sc, int32_t k, V3<R> o, V3<R> d, R t,
                                           V3<R> &p, V3<R> &normal, bool &front) {
  const auto g = sc.geom[k];
  const R inv_r = sc.sh0[k].x;
  p = mk(madd<F>(t, d.x, o.x), madd<F>(t, d.y, o.y), madd<F>(t, d.z, o.z));  // ray::at ray.h:15
  const V3<R> outward = scale(inv_r, mk(p.x - g.x, p.y - g.y, p.z - g.z));
  front = dot<F>(d, outward) < R(0);
  normal = front ? outward : mk(-outward.x, -outward.y, -outward.z);
}

// hit_record for the fast kernels, given the sphere's geom record g and 1/r
// (loaded by the caller with its shade records)
__device__ __forceinline__ void hit_record_fast(const float4 g, float inv_r, V3<float> o, V3<float> d, float t,
                                                V3<float> &p, V3<float> &normal, bool &front) {
  p = mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));  // ray::at ray.h:15
  const V3<float> outward = scale(inv_r, mk(p.x - g.x, p.y - g.y, p.z - g.z));
  front = dot<true>(d, outward) < 0.0f;
  normal = front ? outward : mk(-outward.x, -outward.y, -outward.z);
}

// sky, main.cpp:80-82, given inv_len = 1/sqrt(d.d) (the fast kernels share it)
__device__ __forceinline__ V3<float> sky_fast(V3<float> d, float inv_len) {
  const float uy = inv_len * d.y;
  const float t = 0.5f * (uy + 1.0f);
  return mk(__builtin_fmaf(t, 0.5f, 1.0f - t), __builtin_fmaf(t, 0.7f, 1.0f - t), __builtin_fmaf(t, 1.0f, 1.0f - t));
}
template <bool F, class R> __device__ __forceinline__ V3<R> sky(V3<R> d) {
  const R uy = drcp(dsqrt(dot<F>(d, d))) * d.y;
  const R t = R(0.5) * (uy + R(1));
  return mk(madd<F>(t, R(0.5), R(1) - t), madd<F>(t, R(0.7), R(1) - t), madd<F>(t, R(1), R(1) - t));
}

}  // namespace rtmi
