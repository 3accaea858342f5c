/* oracle/rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 * CPU restatement of rt_in_one_weekend/'s hot path.  Built by oracle/Makefile
 * with -ffp-contract=off: the only fused multiply-adds are the explicit
 * fmaf() calls of the fast policy.  Reference citations are file:line into
 * /root/reference/rt_in_one_weekend/.
 */
#define _GNU_SOURCE
#include "rt_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------- */
/* glibc random_r TYPE_3 (x**31 + x**3 + 1), the generator behind rand()    */
/* (rtweekend.h:21-24).  Restated from glibc's published algorithm          */
/* (stdlib/random_r.c, unchanged since 1995); pinned by the scene fixture   */
/* and the seeded KATs.                                                     */
/* ---------------------------------------------------------------------- */
void or_glibc_seed(or_glibc *g, uint32_t seed) {
  if (seed == 0) seed = 1;
  g->state[0] = (int32_t)seed;
  int32_t word = (int32_t)seed;
  for (int i = 1; i < 31; i++) {
    long hi = word / 127773;
    long lo = word % 127773;
    long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    g->state[i] = word;
  }
  g->f = 3;
  g->r = 0;
  for (int k = 0; k < 310; k++) (void)or_glibc_rand(g);
  g->draws = 0;
}

int32_t or_glibc_rand(or_glibc *g) {
  uint32_t val = (uint32_t)g->state[g->f] + (uint32_t)g->state[g->r];
  g->state[g->f] = (int32_t)val;
  int32_t result = (int32_t)(val >> 1);
  g->f++;
  if (g->f >= 31) {
    g->f = 0;
    g->r++;
  } else {
    g->r++;
    if (g->r >= 31) g->r = 0;
  }
  g->draws++;
  return result;
}

/* random_double() rtweekend.h:21-24 */
static inline double glibc_uni(or_glibc *g) { return (double)or_glibc_rand(g) / (2147483647 + 1.0); }

/* ---------------------------------------------------------------------- */
/* xoroshiro128+ keyed per (seed, pixel, sample): the fast-mode stream.     */
/* ---------------------------------------------------------------------- */
typedef struct xo {
  uint64_t s0, s1;
} xo;

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline void xo_init(xo *g, uint64_t seed, uint64_t pixel, uint32_t sample) {
  uint64_t key = (pixel << 24) | (uint64_t)sample;
  g->s0 = mix64(seed ^ (key * 0x9E3779B97F4A7C15ULL)); /* splitmix64 with the key as counter */
  g->s1 = mix64(g->s0 + 0x9E3779B97F4A7C15ULL);
}
static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xo_next(xo *g) {
  uint64_t s0 = g->s0, s1 = g->s1, r = s0 + s1;
  s1 ^= s0;
  g->s0 = rotl64(s0, 24) ^ s1 ^ (s1 << 16);
  g->s1 = rotl64(s1, 37);
  return r;
}
/* top 24 bits -> [0,1) exactly representable in float */
static inline float xo_uni(xo *g) { return (float)(uint32_t)(xo_next(g) >> 40) * 0x1p-24f; }
/* two uniforms from one step: bits 63..40 and 39..16 */
static inline void xo_pair(xo *g, float *u, float *v) {
  uint64_t r = xo_next(g);
  *u = (float)(uint32_t)(r >> 40) * 0x1p-24f;
  *v = (float)(uint32_t)((r >> 16) & 0xFFFFFFu) * 0x1p-24f;
}
/* cos and sin of 2*pi*v, v in [0,1) a multiple of 2^-24: exact quadrant
 * reduction, then Cephes' sinf/cosf polynomials on [-pi/4, pi/4] with
 * explicit fmaf (the GPU evaluates the identical sequence). */
static inline void sincos2pi(float v, float *c, float *s) {
  const float t = v * 4.0f;
  const int k = (int)(t + 0.5f);
  const float x = (t - (float)k) * 1.57079637f;
  const float x2 = x * x;
  float p = fmaf(x2, -1.9515295891e-4f, 8.3321608736e-3f);
  p = fmaf(x2, p, -1.6666654611e-1f);
  const float sn = fmaf(x * x2, p, x);
  float q = fmaf(x2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  q = fmaf(x2, q, 4.166664568298827e-2f);
  const float cs = fmaf(x2 * x2, q, fmaf(-0.5f, x2, 1.0f));
  switch (k & 3) {
    case 0: *c = cs; *s = sn; break;
    case 1: *c = -sn; *s = cs; break;
    case 2: *c = -cs; *s = -sn; break;
    default: *c = sn; *s = -cs; break;
  }
}

void or_fast_rng(uint64_t seed, uint64_t pixel, uint32_t sample, int32_t n, uint64_t *out) {
  xo g;
  xo_init(&g, seed, pixel, sample);
  for (int32_t i = 0; i < n; i++) out[i] = xo_next(&g);
}

/* ---------------------------------------------------------------------- */
/* ref instantiation: double, no FMA, glibc stream, recursion order.        */
/* ---------------------------------------------------------------------- */
#define RAY_OFFSET 0
#define HIT_EXPANDED 0
#define DIRECT_SAMPLING 0
#define PFX(x) ref_##x
#define R double
#define MADD(a, b, c) ((a) * (b) + (c))
#define SQRT sqrt
#define FMIN fmin
#define FABS fabs
#define POW5(x) pow((x), 5)
#define RNG_T or_glibc
#define UNI(g) glibc_uni(g)
#define ROOT(num, a, ia) ((num) / (a))
#define T_STACK 1
#include "rt_oracle_core.inc"
#undef PFX
#undef R
#undef MADD
#undef SQRT
#undef FMIN
#undef FABS
#undef POW5
#undef RNG_T
#undef UNI
#undef ROOT
#undef T_STACK
#undef RAY_OFFSET
#undef HIT_EXPANDED
#undef DIRECT_SAMPLING

/* ---------------------------------------------------------------------- */
/* fast instantiation: float, fmaf policy, xoroshiro, forward product.      */
/* ---------------------------------------------------------------------- */
static inline float pow5f(float x) {
  float x2 = x * x;
  float x4 = x2 * x2;
  return x4 * x;
}
#define RAY_OFFSET 1
#define HIT_EXPANDED 1
#define DIRECT_SAMPLING 1
#define PFX(x) fast_##x
#define R float
#define MADD(a, b, c) fmaf((a), (b), (c))
#define SQRT sqrtf
#define FMIN fminf
#define FABS fabsf
#define POW5(x) pow5f(x)
#define RNG_T xo
#define UNI(g) xo_uni(g)
#define ROOT(num, a, ia) ((num) * (ia))
#define T_STACK 0
#include "rt_oracle_core.inc"
#undef PFX
#undef R
#undef MADD
#undef SQRT
#undef FMIN
#undef FABS
#undef POW5
#undef RNG_T
#undef UNI
#undef ROOT
#undef T_STACK

/* Test hook: n draws of the fast-mode direct samplers (kind 0: unit
 * direction, 1: point in the unit ball, 2: point in the unit disk) from the
 * stream (seed, pixel 0, sample 0), as xyz triples; 3: (cos, sin, v) of
 * 2 pi v for v = (i * 4099 mod 2^24) * 2^-24 (sincos2pi accuracy). */
void or_fast_dirs(int32_t kind, uint64_t seed, int32_t n, float *out) {
  xo g;
  xo_init(&g, seed, 0, 0);
  for (int32_t i = 0; i < n; i++) {
    fast_V p = {0, 0, 0};
    if (kind == 0) p = fast_unit_dir(&g);
    else if (kind == 1) p = fast_in_sphere_direct(&g);
    else if (kind == 2) p = fast_in_disk_direct(&g);
    else {
      float c, s, v = (float)(((int64_t)i * 4099) & 0xFFFFFF) * 0x1p-24f;
      sincos2pi(v, &c, &s);
      p.x = c; p.y = s; p.z = v;
    }
    out[3 * i] = p.x;
    out[3 * i + 1] = p.y;
    out[3 * i + 2] = p.z;
  }
}

/* ---------------------------------------------------------------------- */
/* Scenes and camera (host, double)                                         */
/* ---------------------------------------------------------------------- */
static void put(double *geom, int32_t *kind, double *mat, int32_t k, double cx, double cy, double cz,
                double r, int32_t kd, double a0, double a1, double a2, double f) {
  geom[4 * k + 0] = cx; geom[4 * k + 1] = cy; geom[4 * k + 2] = cz; geom[4 * k + 3] = r;
  kind[k] = kd;
  mat[4 * k + 0] = a0; mat[4 * k + 1] = a1; mat[4 * k + 2] = a2; mat[4 * k + 3] = f;
}

/* random_scene() main.cpp:86-131, GCC draw order. */
int32_t or_final_scene(or_glibc *g, double *geom, int32_t *kind, double *mat, int32_t cap) {
  int32_t n = 0;
#define PUT(...) do { if (n >= cap) return -1; put(geom, kind, mat, n++, __VA_ARGS__); } while (0)
  PUT(0, -1000, 0, 1000, 0, 0.5, 0.5, 0.5, 0); /* main.cpp:89-90 */
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      double choose_mat = glibc_uni(g);                 /* :94 */
      double rz = glibc_uni(g), rx = glibc_uni(g);      /* :95, right-to-left */
      double cx = a + 0.9 * rx, cy = 0.2, cz = b + 0.9 * rz;
      double dx = cx - 4, dy = cy - 0.2, dz = cz - 0;
      if (sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {    /* :97 */
        if (choose_mat < 0.8) {                         /* :100-104 */
          double bz = glibc_uni(g), by = glibc_uni(g), bx = glibc_uni(g);
          double az = glibc_uni(g), ay = glibc_uni(g), ax = glibc_uni(g);
          PUT(cx, cy, cz, 0.2, 0, ax * bx, ay * by, az * bz, 0);
        } else if (choose_mat < 0.95) {                 /* :105-110 */
          double z = 0.5 + (1 - 0.5) * glibc_uni(g);
          double y = 0.5 + (1 - 0.5) * glibc_uni(g);
          double x = 0.5 + (1 - 0.5) * glibc_uni(g);
          double fuzz = 0 + (0.5 - 0) * glibc_uni(g);
          PUT(cx, cy, cz, 0.2, 1, x, y, z, fuzz < 1 ? fuzz : 1);
        } else {                                        /* :111-114 */
          PUT(cx, cy, cz, 0.2, 2, 0, 0, 0, 1.5);
        }
      }
    }
  }
  PUT(0, 1, 0, 1.0, 2, 0, 0, 0, 1.5);        /* :121-122 */
  PUT(-4, 1, 0, 1.0, 0, 0.4, 0.2, 0.1, 0);   /* :124-125 */
  PUT(4, 1, 0, 1.0, 1, 0.7, 0.6, 0.5, 0.0);  /* :127-128 */
#undef PUT
  return n;
}

/* learn() main.cpp:198-210 */
int32_t or_learn_scene(double *geom, int32_t *kind, double *mat, int32_t cap) {
  if (cap < 5) return -1;
  put(geom, kind, mat, 0, 0, -100.5, -1.0, 100, 0, 0.8, 0.8, 0.0, 0);
  put(geom, kind, mat, 1, 0, 0, -1.0, 0.5, 0, 0.1, 0.2, 0.5, 0);
  put(geom, kind, mat, 2, -1.0, 0, -1.0, 0.5, 2, 0, 0, 0, 1.5);
  put(geom, kind, mat, 3, -1.0, 0.0, -1.0, -0.4, 2, 0, 0, 0, 1.5);
  put(geom, kind, mat, 4, 1.0, 0, -1.0, 0.5, 1, 0.8, 0.6, 0.2, 1.0);
  return 5;
}

/* camera::camera camera.h:8-45 (double, reference op order) */
void or_camera_make(or_camera *c, const double lf[3], const double la[3], const double vup[3],
                    double vfov, double aspect, double aperture, double focus) {
  const double pi = 3.1415926535897932385;
  double theta = vfov * pi / 180.0;
  double h = tan(theta / 2);
  double vh = 2.0 * h, vw = aspect * vh;
  ref_V d = ref_mk(lf[0] - la[0], lf[1] - la[1], lf[2] - la[2]);
  ref_V w = ref_unit(d);
  ref_V up = ref_mk(vup[0], vup[1], vup[2]);
  ref_V cr = ref_mk(up.y * w.z - up.z * w.y, up.z * w.x - up.x * w.z, up.x * w.y - up.y * w.x);
  ref_V u = ref_unit(cr);
  ref_V v = ref_mk(w.y * u.z - w.z * u.y, w.z * u.x - w.x * u.z, w.x * u.y - w.y * u.x);
  ref_V org = ref_mk(lf[0], lf[1], lf[2]);
  ref_V hor = ref_scale(focus * vw, u);
  ref_V ver = ref_scale(focus * vh, v);
  ref_V llc = ref_sub(ref_sub(ref_sub(org, ref_scale(1.0 / 2, hor)), ref_scale(1.0 / 2, ver)), ref_scale(focus, w));
  double *dst[7] = {c->origin, c->lower_left_corner, c->horizontal, c->vertical, c->u, c->v, c->w};
  ref_V src[7] = {org, llc, hor, ver, u, v, w};
  for (int i = 0; i < 7; i++) { dst[i][0] = src[i].x; dst[i][1] = src[i].y; dst[i][2] = src[i].z; }
  c->lens_radius = aperture / 2;
}

/* ---------------------------------------------------------------------- */
/* ref-mode API                                                             */
/* ---------------------------------------------------------------------- */
static int64_t g_ref_last_segments = 0;
int64_t or_ref_last_segments(void) { return g_ref_last_segments; }

int64_t or_ref_worker(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                      int32_t max_depth, int32_t start, int32_t end, or_glibc *g, double *out) {
  ref_world w;
  ref_cam k;
  ref_build_world(s, &w);
  ref_build_cam(c, &k);
  int64_t d0 = g->draws, segs = 0;
  for (int32_t index = start; index < end; index++) { /* main.cpp:273-289 */
    int32_t j = index / W, i = index % W;
    ref_V sum = ref_mk(0, 0, 0);
    for (int32_t q = 0; q < spp; q++) sum = ref_add(sum, ref_sample(&w, &k, W, H, max_depth, i, j, g, &segs));
    double *o = out + 3 * (int64_t)(index - start);
    o[0] = sum.x; o[1] = sum.y; o[2] = sum.z;
  }
  free(w.s);
  g_ref_last_segments = segs;
  return g->draws - d0;
}

int32_t or_ref_kat(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t max_depth,
                   int32_t i, int32_t j, uint32_t seed, double out[3]) {
  ref_world w;
  ref_cam k;
  ref_build_world(s, &w);
  ref_build_cam(c, &k);
  or_glibc g;
  or_glibc_seed(&g, seed);
  int64_t segs = 0;
  ref_V col = ref_sample(&w, &k, W, H, max_depth, i, j, &g, &segs);
  out[0] = col.x; out[1] = col.y; out[2] = col.z;
  free(w.s);
  return or_glibc_rand(&g);
}

int32_t or_ref_sphere_hit(const double center[3], double radius, const double o[3], const double d[3],
                          double t_min, double t_max, double *t, double p[3], double normal[3],
                          int32_t *front_face) {
  ref_sph sp;
  memset(&sp, 0, sizeof sp);
  sp.cx = center[0]; sp.cy = center[1]; sp.cz = center[2]; sp.r = radius;
  sp.rr = radius * radius; sp.inv_r = 1 / radius;
  ref_world w = {1, &sp};
  ref_V ro = ref_mk(o[0], o[1], o[2]), rd = ref_mk(d[0], d[1], d[2]);
  double tt;
  if (ref_hit_world(&w, ro, rd, t_min, t_max, &tt) < 0) return 0;
  ref_V pp = ref_at(ro, tt, rd);
  ref_V outward = ref_scale(sp.inv_r, ref_sub(pp, ref_mk(sp.cx, sp.cy, sp.cz)));
  int front = ref_dot(rd, outward) < 0;
  ref_V n = front ? outward : ref_neg(outward);
  *t = tt;
  p[0] = pp.x; p[1] = pp.y; p[2] = pp.z;
  normal[0] = n.x; normal[1] = n.y; normal[2] = n.z;
  *front_face = front;
  return 1;
}

void or_ref_refract(const double uv[3], const double n[3], double eta, double out[3]) {
  ref_V u = ref_mk(uv[0], uv[1], uv[2]), nn = ref_mk(n[0], n[1], n[2]);
  double cos_theta = fmin(ref_dot(ref_neg(u), nn), 1.0);
  ref_V r = ref_refract(u, nn, eta, cos_theta);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

void or_ref_reflect(const double v[3], const double n[3], double out[3]) {
  ref_V r = ref_reflect(ref_mk(v[0], v[1], v[2]), ref_mk(n[0], n[1], n[2]));
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

double or_ref_reflectance(double cosine, double ref_idx) { return ref_reflectance(cosine, ref_idx); }

int32_t or_ref_near_zero(const double v[3]) { return ref_near_zero(ref_mk(v[0], v[1], v[2])); }

int32_t or_ref_scatter(int32_t kind, const double mat[4], const double din[3], const double p[3],
                       const double normal[3], int32_t front_face, uint32_t seed, double atten[3],
                       double so[3], double sd[3], int32_t *next) {
  ref_sph sp;
  memset(&sp, 0, sizeof sp);
  sp.kind = kind;
  sp.a0 = mat[0]; sp.a1 = mat[1]; sp.a2 = mat[2];
  sp.fuzz = mat[3] < 1 ? mat[3] : 1;
  sp.ir = mat[3];
  sp.inv_ir = 1.0 / mat[3];
  or_glibc g;
  or_glibc_seed(&g, seed);
  ref_V a, d;
  int ok = ref_scatter(&sp, ref_mk(din[0], din[1], din[2]), ref_mk(normal[0], normal[1], normal[2]),
                       front_face, &g, &a, &d);
  atten[0] = a.x; atten[1] = a.y; atten[2] = a.z;
  so[0] = p[0]; so[1] = p[1]; so[2] = p[2];
  sd[0] = d.x; sd[1] = d.y; sd[2] = d.z;
  *next = or_glibc_rand(&g);
  return ok;
}

/* ---------------------------------------------------------------------- */
/* fast-mode API                                                            */
/* ---------------------------------------------------------------------- */
/* per-sample colour -> int64 fixed point, 2^-32 units (truncation) */
/* the kernel's guarded conversion (rtmi_device.hip to_fixed): NaN -> 0,
 * clamped to [0, 64] so the cast is defined and 2^24-sample sums fit (a
 * sample's colour is a product of albedos and sky or emission: non-negative
 * in every scene the reference builds) */
static inline int64_t to_fixed(float c) {
  const float g = c == c ? (c > 64.0f ? 64.0f : (c < 0.0f ? 0.0f : c)) : 0.0f;
  return (int64_t)(g * 4294967296.0f);
}
static inline float from_fixed(int64_t v) { return (float)v * 0x1p-32f; }

static int32_t fast_rows(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                         int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                         int32_t nrows, int64_t *fixed, float *out, int64_t *segs_out) {
  if (W < 2 || H < 2 || spp < 1 || spp >= (1 << 24) || nrows < 0) return -1;
  fast_world w;
  fast_cam k;
  fast_build_world(s, &w);
  fast_build_cam(c, &k);
  int64_t total = (int64_t)nrows * W, segs = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : segs)
  for (int64_t q = 0; q < total; q++) {
    int32_t r = (int32_t)(q / W), i = (int32_t)(q % W);
    int32_t j = row0 + r * row_step;
    int64_t acc[3] = {0, 0, 0};
    if (j >= 0 && j < H) {
      uint64_t pixel = (uint64_t)j * (uint64_t)W + (uint64_t)i;
      for (int32_t smp = 0; smp < spp; smp++) {
        xo g;
        xo_init(&g, seed, pixel, (uint32_t)smp);
        fast_V col = fast_sample(&w, &k, W, H, max_depth, i, j, &g, &segs);
        acc[0] += to_fixed(col.x);
        acc[1] += to_fixed(col.y);
        acc[2] += to_fixed(col.z);
      }
    }
    for (int ch = 0; ch < 3; ch++) {
      if (fixed) fixed[3 * q + ch] = acc[ch];
      if (out) out[3 * q + ch] = from_fixed(acc[ch]);
    }
  }
  free(w.s);
  if (segs_out) *segs_out = segs;
  return 0;
}

int32_t or_fast_render(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                       int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step, int32_t nrows,
                       float *out) {
  return fast_rows(s, c, W, H, spp, max_depth, seed, row0, row_step, nrows, NULL, out, NULL);
}

int32_t or_fast_render_fixed(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                             int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                             int32_t nrows, int64_t *out) {
  return fast_rows(s, c, W, H, spp, max_depth, seed, row0, row_step, nrows, out, NULL, NULL);
}

int64_t or_fast_segments(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                         int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                         int32_t nrows) {
  int64_t segs = 0;
  if (fast_rows(s, c, W, H, spp, max_depth, seed, row0, row_step, nrows, NULL, NULL, &segs) != 0) return -1;
  return segs;
}

int32_t or_fast_sample(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t max_depth,
                       uint64_t seed, int32_t i, int32_t j, int32_t k, float out[3]) {
  fast_world w;
  fast_cam cam;
  fast_build_world(s, &w);
  fast_build_cam(c, &cam);
  xo g;
  xo_init(&g, seed, (uint64_t)j * (uint64_t)W + (uint64_t)i, (uint32_t)k);
  int64_t segs = 0;
  fast_V col = fast_sample(&w, &cam, W, H, max_depth, i, j, &g, &segs);
  out[0] = col.x; out[1] = col.y; out[2] = col.z;
  free(w.s);
  return (int32_t)segs;
}
/* The fast mode's image-plane coordinate (i + r) * (1/D) (fast_sample
 * above; the kernels' camera_ray reads the same reciprocal) against the
 * quotient (i + r) / D of main.cpp:278-279 in float, D = W-1 or H-1, over
 * EVERY numerator the fast path can form: column (row) i in [0, D], jitter
 * r = k 2^-24, k in [0, 2^24) (xo_pair's 24-bit uniforms).  fl(i + r) takes
 * exactly the values k 2^-24 (i = 0) and every float in [1, D + 1] (i >= 1:
 * the float spacing in [i, i+1) is a multiple of 2^-24, and a sum rounded up
 * gives i + 1), so those sets are enumerated instead of the D 2^24 pairs.
 * Returns the largest distance between the two results in ulps; counts the
 * numerators checked and those whose two results differ. */
int32_t or_uv_forms(int32_t D, int64_t *n_checked, int64_t *n_diff) {
  const float d = (float)D, inv = 1.0f / d;
  uint32_t hi_bits;
  {
    const float top = (float)D + 1.0f;
    memcpy(&hi_bits, &top, 4);
  }
  const uint32_t one_bits = 0x3F800000u;
  const int64_t n_low = (int64_t)1 << 24, n_high = (int64_t)(hi_bits - one_bits) + 1;
  int32_t worst = 0;
  int64_t diff = 0;
#pragma omp parallel for schedule(static) reduction(max : worst) reduction(+ : diff)
  for (int64_t q = 0; q < n_low + n_high; q++) {
    float x;
    if (q < n_low) {
      x = (float)q * 0x1p-24f;  /* i = 0 */
    } else {
      const uint32_t b = one_bits + (uint32_t)(q - n_low);
      memcpy(&x, &b, 4);
    }
    const float prod = x * inv, quot = x / d;
    int32_t pb, qb;
    memcpy(&pb, &prod, 4);
    memcpy(&qb, &quot, 4);
    const int32_t dist = pb > qb ? pb - qb : qb - pb;  /* both >= +0: bit distance = ulps */
    if (dist > worst) worst = dist;
    diff += dist != 0;
  }
  if (n_checked) *n_checked = n_low + n_high;
  if (n_diff) *n_diff = diff;
  return worst;
}

#include "rt_nw_oracle.inc"
