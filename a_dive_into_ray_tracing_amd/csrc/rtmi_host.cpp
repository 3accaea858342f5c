// rtmi_host.cpp — host-side half of librtmi.so: error reporting, camera,
// scene construction and PPM output.  No device code; these are the callers
// either side of the kernel and need no GPU.
#include "rtmi_internal.h"

#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace rtmi {

static thread_local std::string g_last_error = "";

int set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

void clear_error() { g_last_error.clear(); }

}  // namespace rtmi

using namespace rtmi;

RTMI_EXPORT const char *rt_last_error(void) { return g_last_error.c_str(); }

RTMI_EXPORT int rt_version(void) { return (RTMI_VERSION_MAJOR << 16) | RTMI_VERSION_MINOR; }

// ---------------------------------------------------------------------------
// camera::camera camera.h:8-45.  Double precision, reference operand order:
// unit_vector(v) = (1/|v|) * v (vec3.h:89,101), x/2 = (1/2)*x.
// ---------------------------------------------------------------------------
namespace {
struct D3 {
  double x, y, z;
};
inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
inline D3 sub(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline D3 scale(double t, D3 v) { return d3(t * v.x, t * v.y, t * v.z); }
inline double len(D3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
inline D3 unit(D3 v) { return scale(1 / len(v), v); }
inline D3 cross(D3 u, D3 v) {
  return d3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
inline void store(double dst[3], D3 v) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; }
}  // namespace

RTMI_EXPORT int rt_camera_init(rt_camera *cam, const double lookfrom[3], const double lookat[3],
                              const double vup[3], double vfov_deg, double aspect_ratio,
                              double aperture, double focus_dist) {
  if (!cam || !lookfrom || !lookat || !vup) return set_error(RT_EINVAL, "rt_camera_init: null argument");
  {  // a camera the reference would build from NaNs is refused instead
    bool finite = std::isfinite(vfov_deg) && std::isfinite(aspect_ratio) && std::isfinite(aperture) &&
                  std::isfinite(focus_dist);
    for (int a = 0; a < 3; ++a) finite = finite && std::isfinite(lookfrom[a]) && std::isfinite(lookat[a]) && std::isfinite(vup[a]);
    const D3 dv = d3(lookfrom[0] - lookat[0], lookfrom[1] - lookat[1], lookfrom[2] - lookat[2]);
    const D3 side = cross(d3(vup[0], vup[1], vup[2]), dv);
    if (!finite || !(vfov_deg > 0 && vfov_deg < 180) || !(aspect_ratio > 0) || aperture < 0 || len(dv) == 0 ||
        len(side) == 0)
      return set_error(RT_EINVAL, "rt_camera_init: degenerate camera (lookfrom == lookat, vup parallel to the "
                                  "view direction, vfov outside (0, 180), aspect <= 0 or a non-finite value)");
  }
  const double pi = 3.1415926535897932385;            // rtweekend.h:16
  double theta = vfov_deg * pi / 180.0;               // degree_to_radians rtweekend.h:19
  double h = std::tan(theta / 2);
  double viewport_height = 2.0 * h;
  double viewport_width = aspect_ratio * viewport_height;
  D3 lf = d3(lookfrom[0], lookfrom[1], lookfrom[2]);
  D3 w = unit(sub(lf, d3(lookat[0], lookat[1], lookat[2])));
  D3 u = unit(cross(d3(vup[0], vup[1], vup[2]), w));
  D3 v = cross(w, u);
  D3 horizontal = scale(focus_dist * viewport_width, u);
  D3 vertical = scale(focus_dist * viewport_height, v);
  D3 llc = sub(sub(sub(lf, scale(1.0 / 2, horizontal)), scale(1.0 / 2, vertical)), scale(focus_dist, w));
  store(cam->origin, lf);
  store(cam->lower_left_corner, llc);
  store(cam->horizontal, horizontal);
  store(cam->vertical, vertical);
  store(cam->u, u);
  store(cam->v, v);
  store(cam->w, w);
  cam->lens_radius = aperture / 2;
  return RT_OK;
}

// ---------------------------------------------------------------------------
// random_scene() main.cpp:86-131.  The reference draws from glibc rand()
// (TYPE_3, default seed 1) and its C++ argument evaluation is right-to-left
// under GCC: point3(a+0.9*rd(), 0.2, b+0.9*rd()) draws z first,
// vec3(rd(),rd(),rd()) draws z, y, x.  The sequence is spelled out here so
// any compiler (this file is built by hipcc/clang) reproduces it.  A private
// random_r state keeps the caller's rand() stream untouched.
// ---------------------------------------------------------------------------
namespace {
struct GlibcStream {
  random_data data;
  char state[128];  // 128 bytes -> TYPE_3, as glibc's default rand()
  explicit GlibcStream(uint32_t seed) {
    std::memset(&data, 0, sizeof data);
    std::memset(state, 0, sizeof state);
    initstate_r(seed, state, sizeof state, &data);
  }
  double next() {  // random_double() rtweekend.h:21-24
    int32_t r;
    random_r(&data, &r);
    return r / (RAND_MAX + 1.0);
  }
};

struct SceneWriter {
  double *g;
  int32_t *k;
  double *m;
  int32_t cap, n = 0;
  bool overflow = false;
  void add(double cx, double cy, double cz, double r, int32_t kind, double a0, double a1, double a2,
           double p) {
    if (n >= cap) { overflow = true; return; }
    g[4 * n + 0] = cx; g[4 * n + 1] = cy; g[4 * n + 2] = cz; g[4 * n + 3] = r;
    k[n] = kind;
    m[4 * n + 0] = a0; m[4 * n + 1] = a1; m[4 * n + 2] = a2; m[4 * n + 3] = p;
    n++;
  }
};
}  // namespace

RTMI_EXPORT int rt_scene_random(uint32_t glibc_seed, double *center_radius, int32_t *mat_kind,
                               double *mat_params, int32_t cap, int32_t *n_out) {
  if (!center_radius || !mat_kind || !mat_params || !n_out || cap < 0)
    return set_error(RT_EINVAL, "rt_scene_random: bad argument");
  GlibcStream rs(glibc_seed);
  SceneWriter w{center_radius, mat_kind, mat_params, cap};
  w.add(0, -1000, 0, 1000, RT_MAT_LAMBERTIAN, 0.5, 0.5, 0.5, 0);  // :89-90
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      const double choose_mat = rs.next();  // :94
      const double rz = rs.next();          // :95 third argument first
      const double rx = rs.next();
      const double cx = a + 0.9 * rx, cy = 0.2, cz = b + 0.9 * rz;
      const double dx = cx - 4, dy = cy - 0.2, dz = cz - 0;
      if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {  // :97
        if (choose_mat < 0.8) {                             // :100-104, albedo = random()*random()
          const double bz = rs.next(), by = rs.next(), bx = rs.next();
          const double az = rs.next(), ay = rs.next(), ax = rs.next();
          w.add(cx, cy, cz, 0.2, RT_MAT_LAMBERTIAN, ax * bx, ay * by, az * bz, 0);
        } else if (choose_mat < 0.95) {  // :105-110, random(0.5,1) then fuzz
          const double z = 0.5 + (1 - 0.5) * rs.next();
          const double y = 0.5 + (1 - 0.5) * rs.next();
          const double x = 0.5 + (1 - 0.5) * rs.next();
          const double fuzz = 0 + (0.5 - 0) * rs.next();
          w.add(cx, cy, cz, 0.2, RT_MAT_METAL, x, y, z, fuzz < 1 ? fuzz : 1);
        } else {  // :111-114
          w.add(cx, cy, cz, 0.2, RT_MAT_DIELECTRIC, 0, 0, 0, 1.5);
        }
      }
    }
  }
  w.add(0, 1, 0, 1.0, RT_MAT_DIELECTRIC, 0, 0, 0, 1.5);     // :121-122
  w.add(-4, 1, 0, 1.0, RT_MAT_LAMBERTIAN, 0.4, 0.2, 0.1, 0);  // :124-125
  w.add(4, 1, 0, 1.0, RT_MAT_METAL, 0.7, 0.6, 0.5, 0.0);      // :127-128
  if (w.overflow) return set_error(RT_EINVAL, "rt_scene_random: cap %d too small", cap);
  *n_out = w.n;
  return RT_OK;
}

RTMI_EXPORT int rt_scene_learn(double *center_radius, int32_t *mat_kind, double *mat_params,
                              int32_t cap, int32_t *n_out) {
  if (!center_radius || !mat_kind || !mat_params || !n_out) return set_error(RT_EINVAL, "rt_scene_learn: null");
  SceneWriter w{center_radius, mat_kind, mat_params, cap};
  w.add(0, -100.5, -1.0, 100, RT_MAT_LAMBERTIAN, 0.8, 0.8, 0.0, 0);  // main.cpp:198,206
  w.add(0, 0, -1.0, 0.5, RT_MAT_LAMBERTIAN, 0.1, 0.2, 0.5, 0);       // :202,207
  w.add(-1.0, 0, -1.0, 0.5, RT_MAT_DIELECTRIC, 0, 0, 0, 1.5);        // :203,208
  w.add(-1.0, 0.0, -1.0, -0.4, RT_MAT_DIELECTRIC, 0, 0, 0, 1.5);     // :209 hollow glass
  w.add(1.0, 0, -1.0, 0.5, RT_MAT_METAL, 0.8, 0.6, 0.2, 1.0);        // :204,210
  if (w.overflow) return set_error(RT_EINVAL, "rt_scene_learn: cap %d too small", cap);
  *n_out = w.n;
  return RT_OK;
}

// ---------------------------------------------------------------------------
// write_color(out, pixel_color, spp) color.h:14-28: sqrt(sum/spp) gamma,
// int(256*clamp(c, 0, 0.999)); rows written top first (main.cpp:346-355).
// ---------------------------------------------------------------------------
static inline int quant(float sum, double scale) {
  double c = std::sqrt(scale * static_cast<double>(sum));
  // clamp rtweekend.h:31-37.  A NaN passes the reference's clamp and its
  // int cast is undefined there; here it is 0 (negative sums give NaN too)
  if (!(c >= 0.0)) c = 0.0;
  if (c > 0.999) c = 0.999;
  return static_cast<int>(256 * c);
}

RTMI_EXPORT int rt_quantize(const float *sum, int32_t W, int32_t H, int32_t spp, uint8_t *rgb) {
  if (!sum || !rgb || W <= 0 || H <= 0 || spp <= 0) return set_error(RT_EINVAL, "rt_quantize: bad argument");
  const double scale = 1.0 / spp;
  size_t o = 0;
  for (int32_t j = H - 1; j >= 0; --j)
    for (int32_t i = 0; i < W; ++i)
      for (int c = 0; c < 3; c++) rgb[o++] = static_cast<uint8_t>(quant(sum[(size_t(j) * W + i) * 3 + c], scale));
  return RT_OK;
}

RTMI_EXPORT int rt_write_ppm(const char *path, const float *sum, int32_t W, int32_t H, int32_t spp,
                            int32_t binary) {
  if (!path || !sum || W <= 0 || H <= 0 || spp <= 0) return set_error(RT_EINVAL, "rt_write_ppm: bad argument");
  std::vector<uint8_t> rgb(size_t(W) * H * 3);
  rt_quantize(sum, W, H, spp, rgb.data());
  const bool to_stdout = std::strcmp(path, "-") == 0;
  FILE *f = to_stdout ? stdout : std::fopen(path, "wb");
  if (!f) return set_error(RT_EIO, "rt_write_ppm: cannot open %s: %s", path, std::strerror(errno));
  bool ok = true;
  if (binary) {
    ok = std::fprintf(f, "P6\n%d %d\n255\n", W, H) > 0 && std::fwrite(rgb.data(), 1, rgb.size(), f) == rgb.size();
  } else {
    ok = std::fprintf(f, "P3\n%d %d\n255\n", W, H) > 0;
    std::string line;
    line.reserve(size_t(W) * 12);
    for (int32_t j = 0; j < H && ok; ++j) {
      line.clear();
      for (int32_t i = 0; i < W; ++i) {
        const uint8_t *p = &rgb[(size_t(j) * W + i) * 3];
        char buf[16];
        int k = std::snprintf(buf, sizeof buf, "%d %d %d\n", p[0], p[1], p[2]);
        line.append(buf, size_t(k));
      }
      ok = std::fwrite(line.data(), 1, line.size(), f) == line.size();
    }
  }
  if (to_stdout) std::fflush(f);
  else if (std::fclose(f) != 0) ok = false;
  return ok ? RT_OK : set_error(RT_EIO, "rt_write_ppm: write to %s failed", path);
}

// The multi-GPU row partition's inverse: strip g holds image
// rows g, g + G, g + 2G, ... (rt_render_rows with row0 = g, row_step = G) in
// nrows rows each; rows >= H are padding.  The reference has no multi-device
// path (its 16 threads write disjoint slots of one img, main.cpp:318-338).
RTMI_EXPORT int rt_unpermute_rows(const float *strips, int32_t n_strips, int32_t nrows, int32_t W, int32_t H,
                                  float *image) {
  if (!strips || !image || n_strips < 1 || nrows < 0 || W < 1 || H < 1)
    return set_error(RT_EINVAL, "rt_unpermute_rows: bad argument");
  if (int64_t(n_strips) * nrows < H)
    return set_error(RT_EINVAL, "rt_unpermute_rows: %d strips of %d rows cannot hold %d rows", n_strips, nrows, H);
  const size_t row = size_t(W) * 3;
  for (int32_t j = 0; j < H; ++j) {
    const int32_t g = j % n_strips, k = j / n_strips;
    std::memcpy(image + size_t(j) * row, strips + (size_t(g) * size_t(nrows) + size_t(k)) * row, row * sizeof(float));
  }
  return RT_OK;
}

// PFM ("PF", 3 channels): the pre-gamma mean sum/spp, little-endian (scale
// -1), rows bottom to top — the PFM row order is the image's own (row 0 =
// bottom, main.cpp:274), so rows go out in index order.  SURVEY §8(c) item 5.
RTMI_EXPORT int rt_write_pfm(const char *path, const float *sum, int32_t W, int32_t H, int32_t spp) {
  if (!path || !sum || W <= 0 || H <= 0 || spp <= 0) return set_error(RT_EINVAL, "rt_write_pfm: bad argument");
  FILE *f = std::fopen(path, "wb");
  if (!f) return set_error(RT_EIO, "rt_write_pfm: cannot open %s: %s", path, std::strerror(errno));
  bool ok = std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H) > 0;
  std::vector<float> row(size_t(W) * 3);
  const float inv = 1.0f / float(spp);
  for (int32_t j = 0; j < H && ok; ++j) {
    const float *src = sum + size_t(j) * W * 3;
    for (size_t k = 0; k < row.size(); ++k) row[k] = src[k] * inv;
    ok = std::fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? RT_OK : set_error(RT_EIO, "rt_write_pfm: write to %s failed", path);
}

// Scene text format (tests/golden/scene_final.txt): an optional first line
// with the sphere count, then one sphere per line
//   cx cy cz r kind a0 a1 a2 p      (kind RT_MAT_*; p = fuzz | ir; %.17g)
// '#' starts a comment.  Values are the constructor arguments of
// sphere(center, r, material) (sphere.h:15-19, material.h), so a double
// survives the round trip exactly.
RTMI_EXPORT int rt_scene_write(const char *path, const rt_scene *scene) {
  if (!path || !scene || scene->n < 0 || (scene->n > 0 && (!scene->center_radius || !scene->mat_kind || !scene->mat_params)))
    return set_error(RT_EINVAL, "rt_scene_write: bad argument");
  FILE *f = std::fopen(path, "w");
  if (!f) return set_error(RT_EIO, "rt_scene_write: cannot open %s: %s", path, std::strerror(errno));
  bool ok = std::fprintf(f, "%d\n", scene->n) > 0;
  for (int32_t i = 0; i < scene->n && ok; ++i) {
    const double *g = scene->center_radius + 4 * i, *m = scene->mat_params + 4 * i;
    ok = std::fprintf(f, "%.17g %.17g %.17g %.17g %d %.17g %.17g %.17g %.17g\n", g[0], g[1], g[2], g[3],
                      scene->mat_kind[i], m[0], m[1], m[2], m[3]) > 0;
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? RT_OK : set_error(RT_EIO, "rt_scene_write: write to %s failed", path);
}

RTMI_EXPORT int rt_scene_read(const char *path, double *center_radius, int32_t *mat_kind, double *mat_params,
                              int32_t cap, int32_t *n_out) {
  if (!path || !n_out || cap < 0 || (cap > 0 && (!center_radius || !mat_kind || !mat_params)))
    return set_error(RT_EINVAL, "rt_scene_read: bad argument");
  FILE *f = std::fopen(path, "r");
  if (!f) return set_error(RT_EIO, "rt_scene_read: cannot open %s: %s", path, std::strerror(errno));
  SceneWriter w{center_radius, mat_kind, mat_params, cap};
  char line[1024];
  int lineno = 0;
  long declared = -1;
  int rc = RT_OK;
  while (std::fgets(line, sizeof line, f)) {
    ++lineno;
    if (char *h = std::strchr(line, '#')) *h = 0;
    double v[9];
    int kind = 0;
    const int got = std::sscanf(line, "%lf %lf %lf %lf %d %lf %lf %lf %lf", &v[0], &v[1], &v[2], &v[3], &kind, &v[5],
                                &v[6], &v[7], &v[8]);
    if (got <= 0) continue;  // blank / comment
    if (got == 1 && declared < 0 && w.n == 0 && !w.overflow) {
      if (!(v[0] >= 0 && v[0] <= 2147483647.0 && v[0] == std::floor(v[0]))) {  // range-checked before the cast
        rc = set_error(RT_EINVAL, "%s:%d: bad sphere count", path, lineno);
        break;
      }
      declared = long(v[0]);
      continue;
    }
    if (got != 9) { rc = set_error(RT_EINVAL, "%s:%d: expected 9 fields, got %d", path, lineno, got); break; }
    if (kind < RT_MAT_LAMBERTIAN || kind > RT_MAT_DIELECTRIC) {
      rc = set_error(RT_EINVAL, "%s:%d: unknown material kind %d", path, lineno, kind);
      break;
    }
    bool finite = true;
    for (int k : {0, 1, 2, 3, 5, 6, 7, 8}) finite = finite && std::isfinite(v[k]);
    if (!finite || v[3] == 0.0) { rc = set_error(RT_EINVAL, "%s:%d: non-finite value or zero radius", path, lineno); break; }
    w.add(v[0], v[1], v[2], v[3], kind, v[5], v[6], v[7], v[8]);
    if (w.overflow) ++w.n;  // keep counting for *n_out
  }
  std::fclose(f);
  if (rc) return rc;
  if (declared >= 0 && declared != w.n)
    return set_error(RT_EINVAL, "%s: header says %ld spheres, file has %d", path, declared, w.n);
  if (w.n == 0) return set_error(RT_EINVAL, "%s: no spheres", path);
  *n_out = w.n;
  if (w.overflow) return set_error(RT_EINVAL, "rt_scene_read: cap %d too small for %d spheres", cap, w.n);
  return RT_OK;
}
