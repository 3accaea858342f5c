/* oracle/rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path (rt_in_one_weekend/, SURVEY
 * §2.2) used solely as the checker by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  The product (librtmi.so) never links it.
 *
 * Two instantiations of one path-tracer body (rt_oracle_core.inc):
 *   ref_*  : double, no FMA, reference op order, glibc TYPE_3 rand() stream,
 *            GCC argument-evaluation order.  Pinned bit-exactly against the
 *            reference's own outputs (tests/golden/, oracle/gen_golden.py).
 *   fast_* : float, explicit fmaf() policy, reciprocal-multiply roots,
 *            forward throughput product, xoroshiro128+ keyed per
 *            (seed, pixel, sample), int64 fixed-point (2^-32) accumulation.
 *            This is the numerics contract the HIP kernel must reproduce
 *            bit-for-bit.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_scene {
  int32_t n;
  const double *geom;   /* 4n: cx cy cz radius              (sphere.h:15-19)   */
  const int32_t *kind;  /* n: 0 lambertian, 1 metal, 2 dielectric             */
  const double *mat;    /* 4n: albedo r g b, fuzz | ir      (material.h)       */
} or_scene;

typedef struct or_camera {
  double origin[3], lower_left_corner[3], horizontal[3], vertical[3], u[3], v[3], w[3];
  double lens_radius;   /* camera.h:64-70 */
} or_camera;

/* glibc random_r TYPE_3 (the default rand() generator), restated. */
typedef struct or_glibc {
  int32_t state[31];
  int32_t f, r;         /* indices of fptr / rptr (random_r.c)  */
  int64_t draws;        /* rand() calls since seeding            */
} or_glibc;

void or_glibc_seed(or_glibc *g, uint32_t seed);        /* srand(seed)       */
int32_t or_glibc_rand(or_glibc *g);                    /* rand()            */

/* random_scene() main.cpp:86-131 from stream g (fresh process: seed 1).
 * Returns the object count (487 for seed 1) or -1 if cap is too small. */
int32_t or_final_scene(or_glibc *g, double *geom, int32_t *kind, double *mat, int32_t cap);
/* learn() scene, main.cpp:198-210 (no draws). Returns 5. */
int32_t or_learn_scene(double *geom, int32_t *kind, double *mat, int32_t cap);
/* camera::camera camera.h:8-45 (double). */
void or_camera_make(or_camera *c, const double lookfrom[3], const double lookat[3],
                    const double vup[3], double vfov, double aspect, double aperture,
                    double focus_dist);

/* ---- ref mode (double, glibc stream) ---------------------------------- */
/* worker(start,end,...) main.cpp:267-290 single-threaded over stream g;
 * out: (end-start)*3 sums.  Returns the number of rand() draws consumed. */
int64_t or_ref_worker(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                      int32_t max_depth, int32_t start, int32_t end, or_glibc *g, double *out);
/* world.hit calls of the last or_ref_worker call (single-threaded). */
int64_t or_ref_last_segments(void);
/* One seeded KAT sample: srand(seed); u,v; get_ray; ray_color.  Writes the
 * colour and returns the next rand() value (main.cpp:278-281). */
int32_t or_ref_kat(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t max_depth,
                   int32_t i, int32_t j, uint32_t seed, double out[3]);
/* Function KATs. */
int32_t or_ref_sphere_hit(const double center[3], double radius, const double o[3],
                          const double d[3], double t_min, double t_max, double *t,
                          double p[3], double normal[3], int32_t *front_face);
void or_ref_refract(const double uv[3], const double n[3], double eta, double out[3]);
void or_ref_reflect(const double v[3], const double n[3], double out[3]);
double or_ref_reflectance(double cosine, double ref_idx);
int32_t or_ref_near_zero(const double v[3]);
/* material::scatter with srand(seed) stream; returns scattered flag, writes
 * attenuation, scattered ray, and the next rand() in *next. */
int32_t or_ref_scatter(int32_t kind, const double mat[4], const double din[3], const double p[3],
                       const double normal[3], int32_t front_face, uint32_t seed,
                       double atten[3], double so[3], double sd[3], int32_t *next);

/* ---- fast mode (float, xoroshiro128+, fixed-point sums) -------------- */
/* Render rows row0, row0+row_step, ... (nrows of them) of a W x H image into
 * out[nrows*W*3] as float sums (strip row r = image row row0 + r*row_step).
 * OpenMP over pixels; results are order independent by construction. */
int32_t or_fast_render(const or_scene *s, const or_camera *c, int32_t W, int32_t H, int32_t spp,
                       int32_t max_depth, uint64_t seed, int32_t row0, int32_t row_step,
                       int32_t nrows, float *out);
/* Same, returning the raw int64 fixed-point sums (2^-32 units). */
int32_t or_fast_render_fixed(const or_scene *s, const or_camera *c, int32_t W, int32_t H,
                             int32_t spp, int32_t max_depth, uint64_t seed, int32_t row0,
                             int32_t row_step, int32_t nrows, int64_t *out);
/* One fast-mode sample (pixel (i,j), sample index k): colour + segments. */
int32_t or_fast_sample(const or_scene *s, const or_camera *c, int32_t W, int32_t H,
                       int32_t max_depth, uint64_t seed, int32_t i, int32_t j, int32_t k,
                       float out[3]);
/* xoroshiro128+ stream for key (seed, pixel, sample): first n raw outputs. */
void or_fast_rng(uint64_t seed, uint64_t pixel, uint32_t sample, int32_t n, uint64_t *out);
/* n draws of the fast-mode direct samplers (kind 0 unit direction, 1 unit
 * ball, 2 unit disk; 3 sincos2pi on a v grid) as xyz triples. */
void or_fast_dirs(int32_t kind, uint64_t seed, int32_t n, float *out);
/* Largest ulp distance between (i + r) * (1/D) and (i + r) / D over every
 * float numerator the fast mode forms (i in [0, D], r a 24-bit uniform). */
int32_t or_uv_forms(int32_t D, int64_t *n_checked, int64_t *n_diff);
/* Total path segments (world.hit calls) of the fast-mode render, for the
 * algorithmic-work accounting of bench.py. */
int64_t or_fast_segments(const or_scene *s, const or_camera *c, int32_t W, int32_t H,
                         int32_t spp, int32_t max_depth, uint64_t seed, int32_t row0,
                         int32_t row_step, int32_t nrows);

#ifdef __cplusplus
}
#endif
#endif
