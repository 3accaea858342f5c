// rtmi_nw_path.h — device-side Next-Week path tracing:
// the reference's rt_next_week/cuda/ hittables, textures and materials as
// float code with an explicit fmaf policy (-ffp-contract=off), restated
// operation for operation by the CPU oracle (oracle/rt_nw_oracle.c), so the
// kernel's images equal the oracle's bit for bit.  Transcendentals (sin,
// log, atan2, acos) are our own polynomial evaluations for the same reason.
// Semantics and deviations: DESIGN.md §9.
#pragma once

#include "rtmi_nw_types.h"
#include "rtmi_path.h"

namespace rtmi {
namespace nw {

using V = V3<float>;

__device__ __forceinline__ V add3(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V sub3(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V mul3(V a, V b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot3(V a, V b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
// ray::at: o + t*d
__device__ __forceinline__ V at3(V o, V d, float t) {
  return mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
}

// ---------------------------------------------------------------------------
// transcendentals (mirrored by oracle/rt_nw_oracle.c)
// ---------------------------------------------------------------------------
// sin(x): quadrant k = rint(x * 2/pi), Cody-Waite reduction with a 3-part
// pi/2 (fma: each product exact), then the Cephes sinf/cosf polynomials.
__device__ __forceinline__ float nw_sinf(float x) {
  const float kf = __builtin_rintf(x * 0.636619747f);
  float r = __builtin_fmaf(-kf, 1.57079637f, x);
  r = __builtin_fmaf(-kf, -4.37113883e-8f, r);
  r = __builtin_fmaf(-kf, -1.77635684e-15f, r);
  const int k = int(kf) & 3;
  const float r2 = r * r;
  float p = __builtin_fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  p = __builtin_fmaf(r2, p, -1.6666654611e-1f);
  const float sn = __builtin_fmaf(r * r2, p, r);
  float q = __builtin_fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  q = __builtin_fmaf(r2, q, 4.166664568298827e-2f);
  const float cs = __builtin_fmaf(r2 * r2, q, __builtin_fmaf(-0.5f, r2, 1.0f));
  return k == 0 ? sn : k == 1 ? cs : k == 2 ? -sn : -cs;
}

// log(x), x > 0 normal: Cephes logf (x = m 2^e, m in [sqrt(.5), sqrt(2)))
__device__ __forceinline__ float nw_logf(float x) {
  const int bits = __float_as_int(x);
  int e = ((bits >> 23) & 255) - 126;
  float m = __int_as_float((bits & 0x7fffff) | 0x3f000000);  // [0.5, 1)
  if (m < 0.707106781f) {
    e -= 1;
    m = m + m;
  }
  m = m - 1.0f;
  const float z = m * m;
  float y = __builtin_fmaf(7.0376836292e-2f, m, -1.1514610310e-1f);
  y = __builtin_fmaf(y, m, 1.1676998740e-1f);
  y = __builtin_fmaf(y, m, -1.2420140846e-1f);
  y = __builtin_fmaf(y, m, 1.4249322787e-1f);
  y = __builtin_fmaf(y, m, -1.6668057665e-1f);
  y = __builtin_fmaf(y, m, 2.0000714765e-1f);
  y = __builtin_fmaf(y, m, -2.4999993993e-1f);
  y = __builtin_fmaf(y, m, 3.3333331174e-1f);
  y = (y * m) * z;
  const float fe = float(e);
  y = __builtin_fmaf(fe, -2.12194440e-4f, y);
  y = __builtin_fmaf(-0.5f, z, y);
  return __builtin_fmaf(fe, 0.693359375f, m + y);
}

// atan(x): Cephes atanf
__device__ __forceinline__ float nw_atanf(float x) {
  const bool neg = x < 0.0f;
  float a = neg ? -x : x, y0 = 0.0f;
  if (a > 2.414213562373095f) {
    y0 = 1.57079637f;
    a = -drcp(a);
  } else if (a > 0.4142135623730950f) {
    y0 = 0.785398185f;
    a = (a - 1.0f) / (a + 1.0f);
  }
  const float z = a * a;
  float p = __builtin_fmaf(8.05374449538e-2f, z, -1.38776856032e-1f);
  p = __builtin_fmaf(p, z, 1.99777106478e-1f);
  p = __builtin_fmaf(p, z, -3.33329491539e-1f);
  const float r = __builtin_fmaf(p * z, a, a) + y0;
  return neg ? -r : r;
}
__device__ __forceinline__ float nw_atan2f(float y, float x) {
  if (x == 0.0f) return y > 0.0f ? 1.57079637f : y < 0.0f ? -1.57079637f : 0.0f;
  const float a = nw_atanf(y / x);
  if (x > 0.0f) return a;
  return y >= 0.0f ? a + 3.14159274f : a - 3.14159274f;
}
__device__ __forceinline__ float nw_acosf(float x) {
  x = __builtin_fminf(__builtin_fmaxf(x, -1.0f), 1.0f);
  return nw_atan2f(dsqrt((1.0f - x) * (1.0f + x)), x);
}

// ---------------------------------------------------------------------------
// scene view
// ---------------------------------------------------------------------------
// The Next-Week grid's descriptor: cell c lists
// refs[cell_start[c]] .. refs[cell_start[c+1]] (16-bit leaf-order slots).
struct NwGridDesc {
  float g0[3], h[3], inv_h[3], g1[3];  // origin, cell size, 1/h, far corner
  int32_t n[3];
  int32_t ncells, nrefs;
  const uint16_t *cell_start;  // ncells + 1
  const uint16_t *refs;
};

struct View {
  const DevObj *obj;  // non-media objects, BVH leaf order
  const int32_t *obj_id;
  const Obj *med;  // media, insertion order (evaluated before the BVH walk)
  const int32_t *med_id;
  int32_t nobj, nmed;
  const Inst *inst;
  const Mat *mat;
  const Tex *tex;
  const float4 *perlin_vec;
  const int32_t *perlin_perm;
  const uint8_t *image_px;
  const Image *image;
  const float4 *nlo, *nhi;  // BVH nodes split into {bmin, skip} and {bmax, leaf} (global memory)
  int32_t nnodes;
  float bg[3];
  int32_t has_media;
  // uniform grid over the objects (RT_NW_ACCEL_GRID): its
  // descriptor (cell_start / refs: global copies) and the objects tested
  // brute force beside it (leaf-order slots)
  NwGridDesc grid;
  const int32_t *gbig;
  int32_t nbig;
};

__device__ __forceinline__ float4 ld4(const float (&g)[4]) { return make_float4(g[0], g[1], g[2], g[3]); }

// instance: world ray -> local ray (translate::hit hittable.h:66-69, then
// rotate_y::hit hittable.h:147-156)
__device__ __forceinline__ void to_local(const Inst &in, V &o, V &d) {
  if (in.flags & 2) o = mk(o.x - in.off[0], o.y - in.off[1], o.z - in.off[2]);
  if (in.flags & 1) {
    o = mk(__builtin_fmaf(in.c, o.x, -(in.s * o.z)), o.y, __builtin_fmaf(in.s, o.x, in.c * o.z));
    d = mk(__builtin_fmaf(in.c, d.x, -(in.s * d.z)), d.y, __builtin_fmaf(in.s, d.x, in.c * d.z));
  }
}
// local point / normal -> world (rotate_y hittable.h:162-170, translate :75)
__device__ __forceinline__ V rot_to_world(const Inst &in, V v) {
  return mk(__builtin_fmaf(in.c, v.x, in.s * v.z), v.y, __builtin_fmaf(-in.s, v.x, in.c * v.z));
}

// ---------------------------------------------------------------------------
// hittables, in the object's local frame; each returns whether a root in the
// reference's interval exists and writes it (and the face of a box)
// ---------------------------------------------------------------------------
// sphere::hit sphere.h:42-77: disc > 0, roots strictly inside (t_min, t_max)
__device__ __forceinline__ bool hit_sphere(V o, V d, V c, float r, float tmin, float tmax, float &t) {
  const V oc = sub3(o, c);
  const float a = dot3(d, d);
  const float b = dot3(oc, d);
  const float cc = dot3(oc, oc) - r * r;
  const float disc = __builtin_fmaf(b, b, -(a * cc));
  if (disc > 0.0f) {
    const float sq = dsqrt(disc);
    float tt = (-b - sq) / a;
    if (tt < tmax && tt > tmin) { t = tt; return true; }
    tt = (-b + sq) / a;
    if (tt < tmax && tt > tmin) { t = tt; return true; }
  }
  return false;
}
// moving_sphere::center moving_sphere.h:44-46
__device__ __forceinline__ float time1_of(const Obj &ob) { return ob.g2[0]; }
__device__ __forceinline__ float time1_of(const DevObj &ob) { return ob.t1; }
template <class O> __device__ __forceinline__ V moving_center(const O &ob, float time) {
  // over [0, 1] (every reference scene) the quotient is exactly `time`: skip the division
  const float t1 = time1_of(ob);
  const float f = (ob.g1[3] == 0.0f && t1 == 1.0f) ? time : (time - ob.g1[3]) / (t1 - ob.g1[3]);
  return mk(__builtin_fmaf(f, ob.g1[0] - ob.g0[0], ob.g0[0]), __builtin_fmaf(f, ob.g1[1] - ob.g0[1], ob.g0[1]),
            __builtin_fmaf(f, ob.g1[2] - ob.g0[2], ob.g0[2]));
}
// moving_sphere::hit moving_sphere.h:48-77: disc >= 0, roots in [t_min, t_max]
__device__ __forceinline__ bool hit_moving(V o, V d, V c, float r, float tmin, float tmax, float &t) {
  const V oc = sub3(o, c);
  const float a = dot3(d, d);
  const float hb = dot3(oc, d);
  const float cc = dot3(oc, oc) - r * r;
  const float disc = __builtin_fmaf(hb, hb, -(a * cc));
  if (disc < 0.0f) return false;
  const float sq = dsqrt(disc);
  float root = (-hb - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-hb + sq) / a;
    if (root < tmin || tmax < root) return false;
  }
  t = root;
  return true;
}
// xy_rect / xz_rect / yz_rect ::hit aarect.h:44-72, 103-131, 160-176.
// axis k = plane normal axis, (a, b) = in-plane axes.
template <int KA, int AA, int BA>
__device__ __forceinline__ bool hit_rect(V o, V d, float a0, float a1, float b0, float b1, float k, float tmin,
                                         float tmax, float &t) {
  const float ok = KA == 0 ? o.x : KA == 1 ? o.y : o.z;
  const float dk = KA == 0 ? d.x : KA == 1 ? d.y : d.z;
  const float tt = (k - ok) / dk;
  if (tt < tmin || tt > tmax) return false;
  const float oa = AA == 0 ? o.x : o.y, da = AA == 0 ? d.x : d.y;
  const float ob = BA == 1 ? o.y : o.z, db = BA == 1 ? d.y : d.z;
  const float x = __builtin_fmaf(tt, da, oa);
  const float y = __builtin_fmaf(tt, db, ob);
  if (x < a0 || x > a1 || y < b0 || y > b1) return false;
  t = tt;
  return true;
}
__device__ __forceinline__ bool hit_rect_kind(int kind, V o, V d, const float4 g, float k, float tmin, float tmax,
                                              float &t) {
  if (kind == kRectXY) return hit_rect<2, 0, 1>(o, d, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
  if (kind == kRectXZ) return hit_rect<1, 0, 2>(o, d, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
  return hit_rect<0, 1, 2>(o, d, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
}
// box::hit box.h:53-56 = hittable_list::hit over its six sides (box.h:37-50,
// hittable_list.h:29-44): the shrinking closest_so_far makes a later side win
// a tie.  Returns the face 0..5 in the reference's side order.
__device__ __forceinline__ int hit_box(V o, V d, const float4 p0, const float4 p1, float tmin, float tmax, float &t) {
  int face = -1;
  float closest = tmax, tt;
  if (hit_rect<2, 0, 1>(o, d, p0.x, p1.x, p0.y, p1.y, p1.z, tmin, closest, tt)) { closest = tt; face = 0; }
  if (hit_rect<2, 0, 1>(o, d, p0.x, p1.x, p0.y, p1.y, p0.z, tmin, closest, tt)) { closest = tt; face = 1; }
  if (hit_rect<1, 0, 2>(o, d, p0.x, p1.x, p0.z, p1.z, p1.y, tmin, closest, tt)) { closest = tt; face = 2; }
  if (hit_rect<1, 0, 2>(o, d, p0.x, p1.x, p0.z, p1.z, p0.y, tmin, closest, tt)) { closest = tt; face = 3; }
  if (hit_rect<0, 1, 2>(o, d, p0.y, p1.y, p0.z, p1.z, p1.x, tmin, closest, tt)) { closest = tt; face = 4; }
  if (hit_rect<0, 1, 2>(o, d, p0.y, p1.y, p0.z, p1.z, p0.x, tmin, closest, tt)) { closest = tt; face = 5; }
  t = closest;
  return face;
}

// The rectangles and boxes of hit_object (objects; media boundaries keep the
// division forms above): the plane parameter as (k - o_k) * inv_d_k with
// inv_d = 1/d per axis — of the world ray, computed once per segment, or of
// an instanced object's local ray — instead of a division per plane (six per
// box test).  The oracle's nw_hit_*_inv are the same expressions.
template <int KA, int AA, int BA>
__device__ __forceinline__ bool hit_rect_inv(V o, V d, V inv, float a0, float a1, float b0, float b1, float k,
                                             float tmin, float tmax, float &t) {
  const float ok = KA == 0 ? o.x : KA == 1 ? o.y : o.z;
  const float ik = KA == 0 ? inv.x : KA == 1 ? inv.y : inv.z;
  const float tt = (k - ok) * ik;
  const float oa = AA == 0 ? o.x : o.y, da = AA == 0 ? d.x : d.y;
  const float ob = BA == 1 ? o.y : o.z, db = BA == 1 ? d.y : d.z;
  const float x = __builtin_fmaf(tt, da, oa);
  const float y = __builtin_fmaf(tt, db, ob);
  const bool hit = !(tt < tmin) & !(tt > tmax) & !(x < a0) & !(x > a1) & !(y < b0) & !(y > b1);
  t = hit ? tt : t;
  return hit;
}
__device__ __forceinline__ bool hit_rect_kind_inv(int kind, V o, V d, V inv, const float4 g, float k, float tmin,
                                                  float tmax, float &t) {
  if (kind == kRectXY) return hit_rect_inv<2, 0, 1>(o, d, inv, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
  if (kind == kRectXZ) return hit_rect_inv<1, 0, 2>(o, d, inv, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
  return hit_rect_inv<0, 1, 2>(o, d, inv, g.x, g.y, g.z, g.w, k, tmin, tmax, t);
}
__device__ __forceinline__ int hit_box_inv(V o, V d, V inv, const float4 p0, const float4 p1, float tmin, float tmax,
                                           float &t) {
  int face = -1;
  float closest = tmax, tt;
  tt = closest;
  // each side's test and the update as compares combined bitwise and selects
  // (no exec-mask branches): Next-Week final scene 291 -> 283 ms at 256 spp,
  // profiles/r03/ab_nw_bitwise.txt
  auto side = [&](bool h, int f) {
    closest = h ? tt : closest;
    face = h ? f : face;
  };
  side(hit_rect_inv<2, 0, 1>(o, d, inv, p0.x, p1.x, p0.y, p1.y, p1.z, tmin, closest, tt), 0);
  side(hit_rect_inv<2, 0, 1>(o, d, inv, p0.x, p1.x, p0.y, p1.y, p0.z, tmin, closest, tt), 1);
  side(hit_rect_inv<1, 0, 2>(o, d, inv, p0.x, p1.x, p0.z, p1.z, p1.y, tmin, closest, tt), 2);
  side(hit_rect_inv<1, 0, 2>(o, d, inv, p0.x, p1.x, p0.z, p1.z, p0.y, tmin, closest, tt), 3);
  side(hit_rect_inv<0, 1, 2>(o, d, inv, p0.y, p1.y, p0.z, p1.z, p1.x, tmin, closest, tt), 4);
  side(hit_rect_inv<0, 1, 2>(o, d, inv, p0.y, p1.y, p0.z, p1.z, p0.x, tmin, closest, tt), 5);
  t = closest;
  return face;
}

// a medium's boundary (sphere, moving sphere or box) over (tmin, tmax)
__device__ __forceinline__ bool hit_boundary(const Obj &ob, V o, V d, float time, float tmin, float tmax, float &t) {
  const int bk = ob.aux & 255;
  if (bk == kSphere) return hit_sphere(o, d, mk(ob.g0[0], ob.g0[1], ob.g0[2]), ob.g0[3], tmin, tmax, t);
  if (bk == kMovingSphere) return hit_moving(o, d, moving_center(ob, time), ob.g0[3], tmin, tmax, t);
  return hit_box(o, d, ld4(ob.g0), ld4(ob.g1), tmin, tmax, t) >= 0;
}
// constant_medium::hit constant_medium.h:41-78: entry t1 (clamped to 0) and
// exit t2 of the boundary; the scattering distance -log(u)/density, drawn
// `samples` times (the last that lands inside the boundary wins, DESIGN.md
// §9.2).  The reference puts the scattering point at the entry t1
// (constant_medium.h:73): make_rec recomputes it.
__device__ __forceinline__ float medium_uniform(uint64_t seg_key, int32_t id, int s);
__device__ __forceinline__ bool hit_medium(const Obj &ob, int32_t id, V o, V d, V dw, float time, uint64_t seg_key,
                                           float &t) {
  float r1, r2;
  const int bk = ob.aux & 255;
  if (bk == kSphere || bk == kMovingSphere) {
    // the two boundary calls (constant_medium.h:44-48) share one quadratic:
    // the same roots, selected as each call's interval test would
    const bool mv = bk == kMovingSphere;
    const V c = mv ? moving_center(ob, time) : mk(ob.g0[0], ob.g0[1], ob.g0[2]);
    const float r = ob.g0[3];
    const V oc = sub3(o, c);
    const float a = dot3(d, d), b = dot3(oc, d), cc = dot3(oc, oc) - r * r;
    const float disc = __builtin_fmaf(b, b, -(a * cc));
    if (mv ? disc < 0.0f : !(disc > 0.0f)) return false;  // hit_moving / hit_sphere
    const float sq = dsqrt(disc);
    const float q1 = (-b - sq) / a, q2 = (-b + sq) / a;
    auto pick = [&](float tmin, float tmax, float &out) {
      if (mv) {  // closed interval, hit_moving
        if (!(q1 < tmin || tmax < q1)) { out = q1; return true; }
        if (!(q2 < tmin || tmax < q2)) { out = q2; return true; }
        return false;
      }
      if (q1 < tmax && q1 > tmin) { out = q1; return true; }  // open interval, hit_sphere
      if (q2 < tmax && q2 > tmin) { out = q2; return true; }
      return false;
    };
    if (!pick(-INFINITY, INFINITY, r1)) return false;
    if (!pick(float(double(r1) + 0.00001), INFINITY, r2)) return false;
  } else {
    if (!hit_boundary(ob, o, d, time, -INFINITY, INFINITY, r1)) return false;
    if (!hit_boundary(ob, o, d, time, float(double(r1) + 0.00001), INFINITY, r2)) return false;
  }
  if (r1 < 0.0f) r1 = 0.0f;
  const float len = dsqrt(dot3(dw, dw));
  const float inside = (r2 - r1) * len;
  const int samples = ob.aux >> 8;
  bool hit = false;
  for (int s = 0; s < samples; ++s) {
    const float hd = ob.g2[3] * nw_logf(medium_uniform(seg_key, id, s));
    if (!(hd > inside)) {
      t = r1 + hd / len;
      hit = true;
    }
  }
  return hit;
}

// per-(segment, medium, sample) uniform in (0, 1]: a counter-based draw, so
// no result depends on the order objects are visited in
__device__ __forceinline__ float medium_uniform(uint64_t seg_key, int32_t id, int s) {
  const uint64_t h = mix64(seg_key ^ (uint64_t(uint32_t(id) + 1u) * 0x9E3779B97F4A7C15ULL) ^
                           (uint64_t(uint32_t(s)) * 0xD1B54A32D192ED03ULL));
  return float(uint32_t(h >> 40) + 1u) * 0x1p-24f;
}

// Executed-work counters of the RTMI_STATS build (per lane, added to
// g_nw_stats when an item ends; rt_nw_debug_counters): the algorithmic FLOP of
// every miss test the walk performs — bench.py NW_FLOP's per-kind counts
// (sphere 18, moving sphere 30, rectangle 6, box 36, +15 for an instance's
// ray transform, a medium 2 x its boundary + 4) plus 25 per BVH node slab
// test or grid-box clip and 5 per grid cell step — and the visits.
struct NwCount {
  unsigned long long flop;
  unsigned nodes, objects, cells;
};
__device__ __forceinline__ unsigned nw_test_flop(int kind, bool inst) {
  const unsigned f = kind == kSphere ? 18u : kind == kMovingSphere ? 30u : kind == kBox ? 36u : 6u;
  return f + (inst ? 15u : 0u);
}

// One non-medium object's hit (world ray in; t_min = 0.001, no upper bound:
// the caller applies the order-independent closest rule).  face: box side.
// invw = 1/dw per axis of the world ray (hit_rect_inv).
// S: a spheres-only scene (rt_nw_ctx_set_scene's check: spheres and moving
// spheres, no instances, no media, solid and checker textures): the other
// kinds' code is compiled out — the same arithmetic for the kinds that remain.
template <bool S = false>
__device__ __forceinline__ bool hit_object(const View &sc, const DevObj &ob, V ow, V dw, V invw, float time,
                                           float &t, int &face) {
  if constexpr (S) {
    if ((ob.ka & 255) == kSphere) return hit_sphere(ow, dw, mk(ob.g0[0], ob.g0[1], ob.g0[2]), ob.g0[3], 0.001f, INFINITY, t);
    return hit_moving(ow, dw, moving_center(ob, time), ob.g0[3], 0.001f, INFINITY, t);
  }
  V o = ow, d = dw;
  const bool local = ob.inst >= 0;
  if (local) to_local(sc.inst[ob.inst], o, d);
  const float tmin = 0.001f;
  const int kind = ob.ka & 255;
  switch (kind) {
    case kSphere: return hit_sphere(o, d, mk(ob.g0[0], ob.g0[1], ob.g0[2]), ob.g0[3], tmin, INFINITY, t);
    case kMovingSphere: return hit_moving(o, d, moving_center(ob, time), ob.g0[3], tmin, INFINITY, t);
    case kRectXY: case kRectXZ: case kRectYZ: {
      const V inv = local ? mk(drcp(d.x), drcp(d.y), drcp(d.z)) : invw;
      return hit_rect_kind_inv(kind, o, d, inv, ld4(ob.g0), ob.g1[0], tmin, INFINITY, t);
    }
    default: {
      const V inv = local ? mk(drcp(d.x), drcp(d.y), drcp(d.z)) : invw;
      face = hit_box_inv(o, d, inv, ld4(ob.g0), ld4(ob.g1), tmin, INFINITY, t);
      return face >= 0;
    }
  }
}

// Closest hit of a segment.  1. Media, in insertion order:
// each one that hits is a candidate and sets its bit in the mask.  2. The
// object BVH (global memory, stackless skip-link walk, slab test clipped to
// [0, best_t]); an object whose twin medium hit is skipped.  The winner is
// the smallest (t, insertion index) pair, so no result depends on the visit
// order.  Returns the winner's index: [0, nobj) an object in leaf order,
// nobj + m medium m; -1 none.
// The BVH nodes live in LDS when they fit (staged per block by the kernel,
// rtmi_nw.hip), otherwise in global memory: the walk is a chain of dependent
// node loads.
// LDS layout (dynamic shared memory): nodes lo[nnodes], hi[nnodes]; then, when
// they fit too, the objects (4 float4 each) and their insertion indices.
extern __shared__ float4 nw_nodes_lds[];
template <bool LDS_NODES, bool LDS_OBJS>
__device__ __forceinline__ int32_t hit_world_nw(const View &sc, V o, V d, float time, uint64_t seg_key, float &best_t,
                                                int &best_face, NwCount *cnt) {
  const float4 *nlo = LDS_NODES ? nw_nodes_lds : sc.nlo;
  const float4 *nhi = LDS_NODES ? nw_nodes_lds + sc.nnodes : sc.nhi;
  const DevObj *objs = LDS_OBJS ? reinterpret_cast<const DevObj *>(nw_nodes_lds + 2 * sc.nnodes) : sc.obj;
  const int32_t *oids = LDS_OBJS ? reinterpret_cast<const int32_t *>(nw_nodes_lds + 2 * sc.nnodes + 3 * sc.nobj) : sc.obj_id;
  best_t = INFINITY;
  int32_t best = -1, best_id = 0x7fffffff;
  best_face = -1;
  uint32_t med_hit = 0;
  const V invw = mk(drcp(d.x), drcp(d.y), drcp(d.z));  // hit_object's planes
  for (int32_t m = 0; m < sc.nmed; ++m) {
    const Obj ob = sc.med[m];
    const int32_t id = sc.med_id[m];
    V lo = o, ld = d;
    if (ob.inst >= 0) to_local(sc.inst[ob.inst], lo, ld);
    float t;
    if constexpr (RTMI_STATS) cnt->flop += 2 * nw_test_flop(ob.aux & 255, false) + 4 + (ob.inst >= 0 ? 15 : 0);
    if (hit_medium(ob, id, lo, ld, d, time, seg_key, t) && !(t < 0.001f)) {
      med_hit |= 1u << m;
      if (t < best_t || (t == best_t && id < best_id)) {
        best_t = t;
        best = sc.nobj + m;
        best_id = id;
      }
    }
  }
  auto safe_inv = [](float v) { return drcp(__builtin_fabsf(v) < 1e-20f ? __builtin_copysignf(1e-20f, v) : v); };
  const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
  const float ox = -o.x * ix, oy = -o.y * iy, oz = -o.z * iz;
  int32_t node = 0;
  while (node < sc.nnodes) {
    const float4 lo = nlo[node], hi = nhi[node];
    const float tx0 = __builtin_fmaf(lo.x, ix, ox), tx1 = __builtin_fmaf(hi.x, ix, ox);
    const float ty0 = __builtin_fmaf(lo.y, iy, oy), ty1 = __builtin_fmaf(hi.y, iy, oy);
    const float tz0 = __builtin_fmaf(lo.z, iz, oz), tz1 = __builtin_fmaf(hi.z, iz, oz);
    const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx0, tx1), __builtin_fminf(ty0, ty1)),
                                        __builtin_fmaxf(__builtin_fminf(tz0, tz1), 0.0f));
    const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx0, tx1), __builtin_fmaxf(ty0, ty1)),
                                       __builtin_fminf(__builtin_fmaxf(tz0, tz1), best_t));
    const bool enter = tnear <= tfar;
    const int32_t leaf = __float_as_int(hi.w);
    if constexpr (RTMI_STATS) {
      cnt->flop += 25;
      cnt->nodes += 1;
    }
    if (enter && leaf >= 0) {
      const int32_t first = leaf >> 4, nleaf = leaf & 15;
      for (int32_t k = first; k < first + nleaf; ++k) {
        const DevObj ob = objs[k];
        const int twin = ob.ka >> 8;
        if (twin > 0 && ((med_hit >> (twin - 1)) & 1u)) continue;  // hidden by its medium
        if constexpr (RTMI_STATS) {
          cnt->flop += nw_test_flop(ob.ka & 255, ob.inst >= 0);
          cnt->objects += 1;
        }
        const int32_t id = oids[k];
        float t;
        int face = -1;
        if (hit_object(sc, ob, o, d, invw, time, t, face) && (t < best_t || (t == best_t && id < best_id))) {
          best_t = t;
          best = k;
          best_id = id;
          best_face = face;
        }
      }
    }
    node = enter ? node + 1 : __float_as_int(lo.w);
  }
  return best;
}

// Grid LDS layout (dynamic shared memory, staged per block): the objects
// (3 float4 each) and their insertion indices, then ncells + 1 uint16 cell
// starts and nrefs uint16 refs (leaf-order slots), then the brute-force
// list (int32, 4-byte aligned).
__host__ __device__ constexpr size_t nw_grid_lds_bytes(int32_t nobj, int32_t ncells, int32_t nrefs, int32_t nbig) {
  return size_t(nobj) * 52 + ((size_t(ncells) + 1 + size_t(nrefs)) * 2 + 3) / 4 * 4 + size_t(nbig) * 4;
}

// Closest hit through the uniform grid (RT_NW_ACCEL_GRID): the media first
// (as hit_world_nw), then the brute-force list, then a 3D-DDA walk over the
// cells the ray crosses inside [0, best_t], testing each cell's objects with
// hit_object and the same order-independent (t, insertion index) rule.  The
// walk stops at the first cell whose exit is at or beyond the closest hit so
// far.  Exact for the reasons of the RTIOW grid: an
// object's hit point — world ray at its t, up to the float error of an
// instance transform — lies inside its box grown by its margin (>= 1e-3 of
// its coordinate scale), so inside a cell that lists it; an object listed in
// several cells gives the same t each time.  The objects' boxes cover the
// whole shutter (moving spheres) and the composed transform (instances).
template <bool S = false>
__device__ __forceinline__ int32_t hit_world_nw_grid(const View &sc, V o, V d, float time, uint64_t seg_key,
                                                     float &best_t, int &best_face, NwCount *cnt) {
  const DevObj *objs = reinterpret_cast<const DevObj *>(nw_nodes_lds);
  const int32_t *oids = reinterpret_cast<const int32_t *>(nw_nodes_lds + 3 * sc.nobj);
  const uint16_t *cs = reinterpret_cast<const uint16_t *>(oids + sc.nobj);
  const NwGridDesc &G = sc.grid;
  const uint16_t *refs = cs + G.ncells + 1;
  const int32_t *big = reinterpret_cast<const int32_t *>(
      reinterpret_cast<const char *>(cs) + ((size_t(G.ncells) + 1 + size_t(G.nrefs)) * 2 + 3) / 4 * 4);
  best_t = INFINITY;
  int32_t best = -1, best_id = 0x7fffffff;
  best_face = -1;
  uint32_t med_hit = 0;
  V invw = mk(0.f, 0.f, 0.f);
  if constexpr (!S) {
    invw = mk(drcp(d.x), drcp(d.y), drcp(d.z));  // hit_object's planes
    for (int32_t m = 0; m < sc.nmed; ++m) {
      const Obj ob = sc.med[m];
      const int32_t id = sc.med_id[m];
      V lo = o, ld = d;
      if (ob.inst >= 0) to_local(sc.inst[ob.inst], lo, ld);
      float t;
      if constexpr (RTMI_STATS) cnt->flop += 2 * nw_test_flop(ob.aux & 255, false) + 4 + (ob.inst >= 0 ? 15 : 0);
      if (hit_medium(ob, id, lo, ld, d, time, seg_key, t) && !(t < 0.001f)) {
        med_hit |= 1u << m;
        if (t < best_t || (t == best_t && id < best_id)) {
          best_t = t;
          best = sc.nobj + m;
          best_id = id;
        }
      }
    }
  }
  auto test = [&](int32_t k) {
    const DevObj ob = objs[k];
    const int twin = ob.ka >> 8;
    if (!S && twin > 0 && ((med_hit >> (twin - 1)) & 1u)) return;  // hidden by its medium
    if constexpr (RTMI_STATS) {
      cnt->flop += nw_test_flop(ob.ka & 255, ob.inst >= 0);
      cnt->objects += 1;
    }
    const int32_t id = oids[k];
    float t;
    int face = -1;
    if (hit_object<S>(sc, ob, o, d, invw, time, t, face) && (t < best_t || (t == best_t && id < best_id))) {
      best_t = t;
      best = k;
      best_id = id;
      best_face = face;
    }
  };
  for (int32_t b = 0; b < sc.nbig; ++b) test(big[b]);
  const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
  const float ox = -o.x * ix, oy = -o.y * iy, oz = -o.z * iz;
  const float bx0 = __builtin_fmaf(G.g0[0], ix, ox), bx1 = __builtin_fmaf(G.g1[0], ix, ox);
  const float by0 = __builtin_fmaf(G.g0[1], iy, oy), by1 = __builtin_fmaf(G.g1[1], iy, oy);
  const float bz0 = __builtin_fmaf(G.g0[2], iz, oz), bz1 = __builtin_fmaf(G.g1[2], iz, oz);
  const float tnear = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(bx0, bx1), __builtin_fminf(by0, by1)),
                                      __builtin_fmaxf(__builtin_fminf(bz0, bz1), 0.0f));
  const float tfar = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(bx0, bx1), __builtin_fmaxf(by0, by1)),
                                     __builtin_fminf(__builtin_fmaxf(bz0, bz1), best_t));
  if constexpr (RTMI_STATS) cnt->flop += 25;  // the grid-box clip
  if (tnear <= tfar) {
    auto cell_of = [&](float p, int ax) {
      const int c = int(__builtin_floorf((p - G.g0[ax]) * G.inv_h[ax]));
      return c < 0 ? 0 : (c >= G.n[ax] ? G.n[ax] - 1 : c);
    };
    int cx = cell_of(__builtin_fmaf(tnear, d.x, o.x), 0);
    int cy = cell_of(__builtin_fmaf(tnear, d.y, o.y), 1);
    int cz = cell_of(__builtin_fmaf(tnear, d.z, o.z), 2);
    // step signs from the culling inverses (safe_inv maps -0.0 to -1e20)
    const int sx = ix >= 0.0f ? 1 : -1, sy = iy >= 0.0f ? 1 : -1, sz = iz >= 0.0f ? 1 : -1;
    auto tface = [&](int c, int s, int ax, float inv, float oo) {
      return __builtin_fmaf(__builtin_fmaf(float(c + (s > 0)), G.h[ax], G.g0[ax]), inv, oo);
    };
    float tnx = tface(cx, sx, 0, ix, ox), tny = tface(cy, sy, 1, iy, oy), tnz = tface(cz, sz, 2, iz, oz);
    int cell = cx + G.n[0] * (cy + G.n[1] * cz);
    const int dcx = sx, dcy = sy * G.n[0], dcz = sz * G.n[0] * G.n[1];
    for (;;) {
      if constexpr (RTMI_STATS) {
        cnt->flop += 5;
        cnt->cells += 1;
      }
      const int e = cs[cell + 1];
      for (int r = cs[cell]; r < e; ++r) test(int32_t(refs[r]));
      const float texit = __builtin_fminf(tnx, __builtin_fminf(tny, tnz));
      if (!(texit < best_t)) break;  // the closest hit so far lies in the cells walked
      if (tnx <= tny && tnx <= tnz) {
        cx += sx;
        if (unsigned(cx) >= unsigned(G.n[0])) break;
        cell += dcx;
        tnx = tface(cx, sx, 0, ix, ox);
      } else if (tny <= tnz) {
        cy += sy;
        if (unsigned(cy) >= unsigned(G.n[1])) break;
        cell += dcy;
        tny = tface(cy, sy, 1, iy, oy);
      } else {
        cz += sz;
        if (unsigned(cz) >= unsigned(G.n[2])) break;
        cell += dcz;
        tnz = tface(cz, sz, 2, iz, oz);
      }
    }
  }
  return best;
}

// ---------------------------------------------------------------------------
// textures (texture.h, perlin.h)
// ---------------------------------------------------------------------------
// perlin::noise perlin.h:30-63 + trilinear_interp perlin.h:114-127
__device__ __forceinline__ float perlin_noise(const View &sc, int32_t pid, V p) {
  const float4 *ranvec = sc.perlin_vec + pid * kPerlinN;
  const int32_t *px = sc.perlin_perm + pid * 3 * kPerlinN, *py = px + kPerlinN, *pz = py + kPerlinN;
  const float fx = __builtin_floorf(p.x), fy = __builtin_floorf(p.y), fz = __builtin_floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  u = (u * u) * __builtin_fmaf(-2.0f, u, 3.0f);
  v = (v * v) * __builtin_fmaf(-2.0f, v, 3.0f);
  w = (w * w) * __builtin_fmaf(-2.0f, w, 3.0f);
  const int i = int(fx), j = int(fy), k = int(fz);
  float accum = 0.0f;
#pragma unroll
  for (int di = 0; di < 2; ++di)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj)
#pragma unroll
      for (int dk = 0; dk < 2; ++dk) {
        const float4 c = ranvec[px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255]];
        const float wi = di ? u : 1.0f - u, wj = dj ? v : 1.0f - v, wk = dk ? w : 1.0f - w;
        const float dd = dot3(mk(c.x, c.y, c.z), mk(u - float(di), v - float(dj), w - float(dk)));
        accum = __builtin_fmaf((wi * wj) * wk, dd, accum);
      }
  return accum;
}
// perlin::turb perlin.h:65-78 (depth 7)
__device__ __forceinline__ float perlin_turb(const View &sc, int32_t pid, V p) {
  float accum = 0.0f, weight = 1.0f;
  for (int i = 0; i < 7; ++i) {
    accum = __builtin_fmaf(weight, perlin_noise(sc, pid, p), accum);
    weight *= 0.5f;
    p = mk(p.x * 2.0f, p.y * 2.0f, p.z * 2.0f);
  }
  return __builtin_fabsf(accum);
}

__device__ __forceinline__ V tex_leaf(const View &sc, const Tex &tx, float u, float v, V p) {
  if (tx.kind == kSolid) return mk(tx.rgb[0], tx.rgb[1], tx.rgb[2]);
  if (tx.kind == kNoise) {  // noise_texture::value texture.h:71-80 (marble)
    const V sp = mk(tx.scale * p.x, tx.scale * p.y, tx.scale * p.z);
    const float f = 0.5f * (1.0f + nw_sinf(__builtin_fmaf(10.0f, perlin_turb(sc, tx.a, sp), tx.scale * p.z)));
    return mk(f, f, f);
  }
  // image_texture::value texture.h:94-120
  const Image im = sc.image[tx.a];
  if (im.w == 0) return mk(0.0f, 1.0f, 1.0f);
  u = __builtin_fminf(__builtin_fmaxf(u, 0.0f), 1.0f);
  v = 1.0f - __builtin_fminf(__builtin_fmaxf(v, 0.0f), 1.0f);
  int i = int(u * float(im.w)), j = int(v * float(im.h));
  if (i >= im.w) i = im.w - 1;
  if (j >= im.h) j = im.h - 1;
  i = (i + im.w / 2 + im.w / 3) % im.w;  // "try to shift the map" texture.h:110
  const uint8_t *px = sc.image_px + im.offset + (j * im.w + i) * 3;
  const float s = 1.0f / 255.0f;
  return mk(s * float(px[0]), s * float(px[1]), s * float(px[2]));
}
// texture value; checker_texture::value texture.h:48-55 selects by the sign
// of sin(10x) sin(10y) sin(10z)
template <bool S = false>
__device__ __forceinline__ V tex_value(const View &sc, int32_t tid, float u, float v, V p) {
  Tex tx = sc.tex[tid];
  if (tx.kind == kChecker) {
    const float sines = (nw_sinf(10.0f * p.x) * nw_sinf(10.0f * p.y)) * nw_sinf(10.0f * p.z);
    tx = sc.tex[sines < 0.0f ? tx.b : tx.a];
  }
  if constexpr (S) return mk(tx.rgb[0], tx.rgb[1], tx.rgb[2]);  // (solid leaves only)
  return tex_leaf(sc, tx, u, v, p);
}
__device__ __forceinline__ bool tex_needs_uv(const View &sc, int32_t tid) {
  const Tex tx = sc.tex[tid];
  if (tx.kind == kImage) return true;
  if (tx.kind == kChecker) return sc.tex[tx.a].kind == kImage || sc.tex[tx.b].kind == kImage;
  return false;
}

// sphere::get_sphere_uv sphere.h:30-40
__device__ __forceinline__ void sphere_uv(V p, float &u, float &v) {
  const float theta = nw_acosf(-p.y);
  const float phi = nw_atan2f(-p.z, p.x) + 3.14159274f;
  u = phi / (2.0f * 3.14159274f);
  v = theta / 3.14159274f;
}

// ---------------------------------------------------------------------------
// hit record of the winning object (deferred: recomputed once per segment)
// ---------------------------------------------------------------------------
struct Rec {
  V p, n;
  float u, v;
  int32_t mat;
};
// constant_medium.h:73-77: p at the entry point, arbitrary normal
__device__ __forceinline__ Rec make_rec_medium(const View &sc, const Obj &ob, V ow, V dw, float time) {
  Rec r;
  r.mat = ob.mat;
  r.u = 0.0f;
  r.v = 0.0f;
  V o = ow, d = dw;
  if (ob.inst >= 0) to_local(sc.inst[ob.inst], o, d);
  float r1;
  (void)hit_boundary(ob, o, d, time, -INFINITY, INFINITY, r1);
  if (r1 < 0.0f) r1 = 0.0f;
  r.p = at3(ow, dw, r1);
  r.n = mk(1.0f, 0.0f, 0.0f);
  return r;
}
template <bool S = false>
__device__ __forceinline__ Rec make_rec(const View &sc, const DevObj &ob, V ow, V dw, float time, float t, int face) {
  Rec r;
  r.mat = ob.mat;
  r.u = 0.0f;
  r.v = 0.0f;
  if constexpr (S) {  // a sphere, no instance, no texture reads u, v
    const V c = (ob.ka & 255) == kSphere ? mk(ob.g0[0], ob.g0[1], ob.g0[2]) : moving_center(ob, time);
    const float inv_r = drcp(ob.g0[3]);
    const V p = at3(ow, dw, t);
    r.n = mk(inv_r * (p.x - c.x), inv_r * (p.y - c.y), inv_r * (p.z - c.z));
    r.p = p;
    return r;
  }
  V o = ow, d = dw;
  Inst in{1.f, 0.f, {0.f, 0.f, 0.f}, 0, {0, 0}};
  if (ob.inst >= 0) {
    in = sc.inst[ob.inst];
    to_local(in, o, d);
  }
  V p = at3(o, d, t), n;
  const Mat mm = sc.mat[ob.mat];
  const bool need_uv = mm.kind != kDielectric && tex_needs_uv(sc, mm.tex);
  const int okind = ob.ka & 255;
  if (okind == kSphere || okind == kMovingSphere) {
    const V c = okind == kSphere ? mk(ob.g0[0], ob.g0[1], ob.g0[2]) : moving_center(ob, time);
    const float inv_r = drcp(ob.g0[3]);
    n = mk(inv_r * (p.x - c.x), inv_r * (p.y - c.y), inv_r * (p.z - c.z));
    if (need_uv) sphere_uv(n, r.u, r.v);
  } else {
    int kind = okind;
    float a0, a1, b0, b1;
    if (kind == kBox) {  // box face -> its rect (box.h:37-48)
      const float4 p0 = ld4(ob.g0), p1 = ld4(ob.g1);
      kind = face < 2 ? kRectXY : face < 4 ? kRectXZ : kRectYZ;
      if (kind == kRectXY) { a0 = p0.x; a1 = p1.x; b0 = p0.y; b1 = p1.y; }
      else if (kind == kRectXZ) { a0 = p0.x; a1 = p1.x; b0 = p0.z; b1 = p1.z; }
      else { a0 = p0.y; a1 = p1.y; b0 = p0.z; b1 = p1.z; }
    } else {
      a0 = ob.g0[0]; a1 = ob.g0[1]; b0 = ob.g0[2]; b1 = ob.g0[3];
    }
    // u, v from the in-plane hit coordinates (aarect.h:59-60, 119-120, 170-171)
    float x, y;
    if (kind == kRectXY) { x = __builtin_fmaf(t, d.x, o.x); y = __builtin_fmaf(t, d.y, o.y); n = mk(0.f, 0.f, 1.f); }
    else if (kind == kRectXZ) { x = __builtin_fmaf(t, d.x, o.x); y = __builtin_fmaf(t, d.z, o.z); n = mk(0.f, 1.f, 0.f); }
    else { x = __builtin_fmaf(t, d.y, o.y); y = __builtin_fmaf(t, d.z, o.z); n = mk(1.f, 0.f, 0.f); }
    r.u = (x - a0) / (a1 - a0);
    r.v = (y - b0) / (b1 - b0);
  }
  if (in.flags & 1) {
    p = rot_to_world(in, p);
    n = rot_to_world(in, n);
  }
  if (in.flags & 2) p = mk(p.x + in.off[0], p.y + in.off[1], p.z + in.off[2]);
  r.p = p;
  r.n = n;
  return r;
}

// ---------------------------------------------------------------------------
// materials (rt_next_week/cuda/material.h)
// ---------------------------------------------------------------------------
// schlick material.h:97-101
__device__ __forceinline__ float schlick(float cosine, float ri) {
  float r0 = (1.0f - ri) / (1.0f + ri);
  r0 = r0 * r0;
  return __builtin_fmaf(1.0f - r0, pow5(1.0f - cosine), r0);
}
// Returns true if the ray scattered (dir, atten set); emitted light is
// handled by the caller.
template <bool S = false>
__device__ __forceinline__ bool scatter_nw(const View &sc, const Rec &rec, V din, Xoro &g, V &atten, V &dir) {
  const Mat m = sc.mat[rec.mat];
  switch (m.kind) {
    case kLambertian: {  // material.h:45-55: target = p + n + random_in_unit_sphere
      const V rs = in_sphere_direct(g);
      const V target = add3(add3(rec.p, rec.n), rs);
      dir = sub3(target, rec.p);
      atten = tex_value<S>(sc, m.tex, rec.u, rec.v, rec.p);
      return true;
    }
    case kMetal: {  // material.h:72-86
      const V refl = reflect<true>(unit<true>(din), rec.n);
      const V rs = in_sphere_direct(g);
      dir = mk(__builtin_fmaf(m.fuzz, rs.x, refl.x), __builtin_fmaf(m.fuzz, rs.y, refl.y),
               __builtin_fmaf(m.fuzz, rs.z, refl.z));
      atten = tex_value<S>(sc, m.tex, rec.u, rec.v, rec.p);
      return dot3(dir, rec.n) > 0.0f;
    }
    case kDielectric: {  // material.h:119-148 (+ refract :103-114)
      const V n = rec.n;
      const V reflected = reflect<true>(din, n);
      atten = mk(1.0f, 1.0f, 1.0f);
      const float dn = dot3(din, n);
      const float dlen = dsqrt(dot3(din, din));
      V outward;
      float ni, cosine;
      if (dn > 0.0f) {
        outward = mk(-n.x, -n.y, -n.z);
        ni = m.ir;
        cosine = dn / dlen;
        cosine = dsqrt(1.0f - (m.ir * m.ir) * __builtin_fmaf(-cosine, cosine, 1.0f));
      } else {
        outward = n;
        ni = drcp(m.ir);
        cosine = -dn / dlen;
      }
      const V uv = unit<true>(din);
      const float dt = dot3(uv, outward);
      const float disc = 1.0f - (ni * ni) * __builtin_fmaf(-dt, dt, 1.0f);
      V refracted = mk(0.f, 0.f, 0.f);
      float reflect_prob = 1.0f;
      if (disc > 0.0f) {
        const float sq = dsqrt(disc);
        refracted = mk(__builtin_fmaf(-outward.x, sq, ni * __builtin_fmaf(-outward.x, dt, uv.x)),
                       __builtin_fmaf(-outward.y, sq, ni * __builtin_fmaf(-outward.y, dt, uv.y)),
                       __builtin_fmaf(-outward.z, sq, ni * __builtin_fmaf(-outward.z, dt, uv.z)));
        reflect_prob = schlick(cosine, m.ir);
      }
      dir = g.uni() < reflect_prob ? reflected : refracted;
      return true;
    }
    case kIsotropic: {  // material.h:180-190
      dir = in_sphere_direct(g);
      atten = tex_value<S>(sc, m.tex, rec.u, rec.v, rec.p);
      return true;
    }
    default: return false;  // diffuse_light material.h:159-177
  }
}

}  // namespace nw
}  // namespace rtmi
