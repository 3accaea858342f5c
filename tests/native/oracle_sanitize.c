/* oracle_sanitize.c — TEST INFRASTRUCTURE: drives the oracle (the checker,
 * oracle/rt_oracle.c) under ASan + UBSan, and its OpenMP fast mode under
 * ThreadSanitizer (oracle/Makefile targets asan / tsan; tests/test_sanitize.py).
 * Small renders in ref and fast mode, the function KATs' entry points, the
 * NaN/inf guard and the RNG helpers.  Exit 0 = every check passed and the
 * sanitizers reported nothing (they abort on the first report). */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../oracle/rt_oracle.h"

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

int main(void) {
  static double g[4 * 600], m[4 * 600];
  static int32_t k[600];
  or_glibc rs;
  or_glibc_seed(&rs, 1);
  const int32_t n = or_final_scene(&rs, g, k, m, 600);
  CHECK(n == 487);
  CHECK(or_final_scene(&rs, g, k, m, 10) == -1);
  or_scene sc = {n, g, k, m};
  or_camera cam;
  const double lf[3] = {13, 2, 3}, la[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  or_camera_make(&cam, lf, la, up, 20, 1.5, 0.1, 10);
  /* fast mode, OpenMP over pixels (TSan build: data races would be reported) */
  enum { W = 24, H = 16, S = 4 };
  static float out[W * H * 3];
  CHECK(or_fast_render(&sc, &cam, W, H, S, 50, 1984, 0, 1, H, out) == 0);
  static float strip[5 * W * 3];
  CHECK(or_fast_render(&sc, &cam, W, H, S, 50, 1984, 3, 4, 5, strip) == 0);  /* rows 3..19: past H zero-filled */
  for (int r = 0; r < 4; ++r) CHECK(memcmp(strip + r * W * 3, out + (3 + 4 * r) * W * 3, sizeof(float) * W * 3) == 0);
  for (int i = 0; i < W * 3; ++i) CHECK(strip[4 * W * 3 + i] == 0.0f);
  static int64_t fx[W * H * 3];
  CHECK(or_fast_render_fixed(&sc, &cam, W, H, S, 50, 1984, 0, 1, H, fx) == 0);
  CHECK(or_fast_segments(&sc, &cam, W, H, S, 50, 1984, 0, 1, H) > W * H * S);
  float one[3];
  CHECK(or_fast_sample(&sc, &cam, W, H, 50, 1984, 3, 4, 0, one) >= 1);
  /* ref mode: a few pixels single-threaded from the glibc stream */
  static double ref[8 * 3];
  or_glibc_seed(&rs, 7);
  CHECK(or_ref_worker(&sc, &cam, W, H, 2, 50, 100, 108, &rs, ref) > 0);
  for (int i = 0; i < 24; ++i) CHECK(isfinite(ref[i]) && ref[i] >= 0);
  double kat[3];
  (void)or_ref_kat(&sc, &cam, W, H, 50, 5, 6, 3, kat);
  /* function entry points */
  const double c0[3] = {0, 0, -1}, o[3] = {0, 0, 0}, d[3] = {0, 0, -1};
  double t, p[3], nrm[3];
  int32_t front;
  CHECK(or_ref_sphere_hit(c0, 0.5, o, d, 0.001, INFINITY, &t, p, nrm, &front) == 1 && t == 0.5);
  CHECK(or_ref_sphere_hit(c0, -0.4, o, d, 0.001, INFINITY, &t, p, nrm, &front) == 1);
  double rr[3];
  or_ref_refract(d, nrm, 1.5, rr);
  or_ref_reflect(d, nrm, rr);
  CHECK(or_ref_reflectance(0.5, 1.5) > 0);
  const double z[3] = {0, 0, 0};
  CHECK(or_ref_near_zero(z) == 1);
  double at[3], so[3], sd[3];
  int32_t nx;
  const double mat[4] = {0.5, 0.5, 0.5, 0.3};
  for (int kind = 0; kind < 3; ++kind) (void)or_ref_scatter(kind, mat, d, p, nrm, 1, 11, at, so, sd, &nx);
  uint64_t rng[8];
  or_fast_rng(1984, 12345, 7, 8, rng);
  static float dirs[4 * 300 * 3];
  for (int kind = 0; kind < 4; ++kind) or_fast_dirs(kind, 5, 300, dirs + kind * 900);
  /* non-finite path colours: the guarded fixed-point conversion */
  static double g2[4 * 8], m2[4 * 8];
  static int32_t k2[8];
  const int32_t n2 = or_learn_scene(g2, k2, m2, 8);
  m2[4 * 1 + 0] = NAN;
  m2[4 * 4 + 0] = m2[4 * 4 + 1] = m2[4 * 4 + 2] = 1e30;
  or_scene s2 = {n2, g2, k2, m2};
  or_camera c2;
  const double lf2[3] = {3, 3, 2}, la2[3] = {0, 0, -1};
  or_camera_make(&c2, lf2, la2, up, 20, 16.0 / 9.0, 0.5, sqrt(9 + 9 + 9));
  static float o2[16 * 9 * 3];
  CHECK(or_fast_render(&s2, &c2, 16, 9, 4, 50, 1984, 0, 1, 9, o2) == 0);
  for (int i = 0; i < 16 * 9 * 3; ++i) CHECK(isfinite(o2[i]));
  if (failures) fprintf(stderr, "%d check(s) failed\n", failures);
  else printf("oracle_sanitize: all checks passed\n");
  return failures ? 1 : 0;
}
