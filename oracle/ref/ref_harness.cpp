// oracle/ref/ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference program rt_in_one_weekend/ (compiled from the sources
// where they lie under /root/reference, never copied) so its own functions
// produce the golden vectors committed under tests/golden/ and the timed CPU
// baseline that bench.py reports as cpu_baseline.kind = "reference".
//
// Built by oracle/Makefile into oracle/_ref/ (git-ignored) with g++ — never
// clang/hipcc: the reference's scene depends on GCC's right-to-left argument
// evaluation order.  Nothing in the product links or runs this.
//
// The reference's main() is renamed so this file can provide its own; the
// private static dielectric::reflectance (material.h:91-96) is opened up for
// the function KATs.  Standard headers are included first so the
// `private -> public` rename only reaches the reference's own classes.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <limits>
#include <memory>
#include <string>
#include <thread>
#include <vector>
#include <time.h>

#define main ref_main
#define private public
#include REF_MAIN_CPP
#undef private
#undef main

namespace {

// Tiny private LCG for choosing KAT pixels / function inputs: keeps the
// reference's global rand() stream untouched.
struct Lcg {
  uint64_t s;
  explicit Lcg(uint64_t seed) : s(seed * 6364136223846793005ULL + 1442695040888963407ULL) {}
  uint32_t next() {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return static_cast<uint32_t>(s >> 33);
  }
  double uni() { return next() / 2147483648.0; }             // [0,1)
  double range(double a, double b) { return a + (b - a) * uni(); }
};

void p17(double x) { std::printf(" %.17g", x); }
void pvec(const vec3 &v) { p17(v.x()); p17(v.y()); p17(v.z()); }

// Material of an object as (kind, a0, a1, a2, param); kind 0=L, 1=M, 2=D.
void material_row(const shared_ptr<material> &m, int *kind, double p[4]) {
  p[0] = p[1] = p[2] = p[3] = 0.0;
  if (auto l = std::dynamic_pointer_cast<lambertian>(m)) {
    *kind = 0; p[0] = l->albedo.x(); p[1] = l->albedo.y(); p[2] = l->albedo.z();
  } else if (auto me = std::dynamic_pointer_cast<metal>(m)) {
    *kind = 1; p[0] = me->albedo.x(); p[1] = me->albedo.y(); p[2] = me->albedo.z(); p[3] = me->fuzz;
  } else if (auto d = std::dynamic_pointer_cast<dielectric>(m)) {
    *kind = 2; p[3] = d->ir;
  } else {
    *kind = -1;
  }
}

void dump_world(const hittable_list &world) {
  std::printf("%zu\n", world.objects.size());
  for (const auto &o : world.objects) {
    auto s = std::dynamic_pointer_cast<sphere>(o);
    int kind; double p[4];
    material_row(s->mat_ptr, &kind, p);
    std::printf("%.17g %.17g %.17g %.17g %d %.17g %.17g %.17g %.17g\n", s->center.x(), s->center.y(),
                s->center.z(), s->radius, kind, p[0], p[1], p[2], p[3]);
  }
}

// learn() scene, main.cpp:193-210, built without touching rand().
hittable_list learn_world() {
  hittable_list world;
  auto material_ground = make_shared<lambertian>(color(0.8, 0.8, 0.0));
  auto material_center = make_shared<lambertian>(color(0.1, 0.2, 0.5));
  auto material_left = make_shared<dielectric>(1.5);
  auto material_right = make_shared<metal>(color(0.8, 0.6, 0.2), 1.0);
  world.add(make_shared<sphere>(point3(0, -100.5, -1.0), 100, material_ground));
  world.add(make_shared<sphere>(point3(0, 0, -1.0), 0.5, material_center));
  world.add(make_shared<sphere>(point3(-1.0, 0, -1.0), 0.5, material_left));
  world.add(make_shared<sphere>(point3(-1.0, 0.0, -1.0), -0.4, material_left));
  world.add(make_shared<sphere>(point3(1.0, 0, -1.0), 0.5, material_right));
  return world;
}

// Cameras exactly as the reference builds them (main.cpp:304-311, 212-221).
camera final_camera(double aspect) {
  return camera(point3(13, 2, 3), point3(0, 0, 0), vec3(0, 1, 0), 20, aspect, 0.1, 10.0);
}
camera learn_camera(double aspect) {
  point3 lookfrom(3, 3, 2), lookat(0, 0, -1);
  return camera(lookfrom, lookat, vec3(0, 1, 0), 20, aspect, 0.5, (lookfrom - lookat).length());
}

void dump_camera(const camera &c) {
  std::printf("origin"); pvec(c.origin); std::printf("\n");
  std::printf("lower_left_corner"); pvec(c.lower_left_corner); std::printf("\n");
  std::printf("horizontal"); pvec(c.horizontal); std::printf("\n");
  std::printf("vertical"); pvec(c.vertical); std::printf("\n");
  std::printf("u"); pvec(c.u); std::printf("\n");
  std::printf("v"); pvec(c.v); std::printf("\n");
  std::printf("w"); pvec(c.w); std::printf("\n");
  std::printf("lens_radius"); p17(c.lens_radius); std::printf("\n");
}

bool is_final(const std::string &s) { return s == "final"; }

// Seeded single-sample path KATs: srand(k); the worker()'s per-sample body
// (main.cpp:278-281) for pixel (i,j); print the colour and the next rand().
void kats(const std::string &scene, int n) {
  const bool fin = is_final(scene);
  hittable_list world = fin ? random_scene() : learn_world();
  const int W = fin ? 1200 : 400;
  const int H = fin ? 800 : 225;
  camera cam = fin ? final_camera(3.0 / 2.0) : learn_camera(16.0 / 9.0);
  Lcg pick(fin ? 17 : 29);
  std::printf("%d %d %d\n", n, W, H);
  for (int k = 1; k <= n; k++) {
    int i = static_cast<int>(pick.next() % W);
    int j = static_cast<int>(pick.next() % H);
    srand(static_cast<unsigned>(k));
    auto u = (i + random_double()) / (W - 1);
    auto v = (j + random_double()) / (H - 1);
    ray r = cam.get_ray(u, v);
    color c = ray_color(r, world, 50);
    int next = rand();
    std::printf("%d %d %d", k, i, j);
    pvec(c);
    std::printf(" %d\n", next);
  }
}

// Single-threaded render through the reference worker() (main.cpp:267-290):
// fresh process stream (seed 1), scene first (final consumes draws), then
// every pixel's samples in worker order.  Sums are written as raw little-
// endian float64, W*H*3, index j*W+i, row 0 = bottom.
void image(const std::string &scene, int W, int H, int spp, int depth, const char *out_path) {
  const bool fin = is_final(scene);
  hittable_list world = fin ? random_scene() : learn_world();
  camera cam = fin ? final_camera(double(W) / double(H)) : learn_camera(double(W) / double(H));
  const int size = W * H;
  std::vector<shared_ptr<color>> img(size);
  worker(0, size, std::ref(img), W, H, world, cam, spp, depth);
  std::vector<double> sums(static_cast<size_t>(size) * 3);
  for (int p = 0; p < size; p++) {
    sums[3 * p + 0] = img[p]->x();
    sums[3 * p + 1] = img[p]->y();
    sums[3 * p + 2] = img[p]->z();
  }
  FILE *f = std::fopen(out_path, "wb");
  if (!f) { std::perror(out_path); std::exit(2); }
  std::fwrite(sums.data(), sizeof(double), sums.size(), f);
  std::fclose(f);
  // The reference's own P3 output loop (main.cpp:344-355) on stdout.
  std::cout << "P3\n" << W << ' ' << H << "\n255\n";
  for (int j = H - 1; j >= 0; --j)
    for (int i = 0; i < W; ++i) write_color(std::cout, *img[j * W + i], spp);
}

// Function KATs: sphere::hit, reflect, refract, reflectance, near_zero and
// the three scatter() implementations (srand(k) stream).
void funcs(int n) {
  Lcg g(4242);
  // sphere::hit (sphere.h:21-55) — includes negative radius and finite t_max.
  std::printf("hit %d\n", n);
  for (int k = 0; k < n; k++) {
    point3 c(g.range(-2, 2), g.range(-2, 2), g.range(-2, 2));
    double rad = g.range(0.2, 1.5) * ((k % 5 == 4) ? -1.0 : 1.0);
    if (k % 7 == 6) rad = 1000.0, c = point3(0, -1000, 0);
    point3 o(g.range(-3, 3), g.range(-3, 3), g.range(-3, 3));
    if (k % 4 == 3) o = c + vec3(g.range(-0.1, 0.1), g.range(-0.1, 0.1), g.range(-0.1, 0.1));  // inside
    // aim near the centre so roughly half the rays hit
    vec3 d = (c - o) + vec3(g.range(-1.5, 1.5), g.range(-1.5, 1.5), g.range(-1.5, 1.5));
    if (k % 3 == 2) d = d * g.range(0.1, 4.0);  // unnormalised lengths
    double tmax = (k % 6 == 5) ? g.range(0.5, 3.0) : infinity;
    sphere s(c, rad, make_shared<lambertian>(color(0.5, 0.5, 0.5)));
    hit_record rec;
    rec.t = 0; rec.front_face = false;
    bool h = s.hit(ray(o, d), 0.001, tmax, rec);
    pvec(c); p17(rad); pvec(o); pvec(d); p17(tmax);
    std::printf(" %d", h ? 1 : 0);
    if (h) { p17(rec.t); pvec(rec.p); pvec(rec.normal); std::printf(" %d", rec.front_face ? 1 : 0); }
    std::printf("\n");
  }
  std::printf("refract %d\n", n);
  for (int k = 0; k < n; k++) {
    vec3 uv = unit_vector(vec3(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1)));
    vec3 nn = unit_vector(vec3(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1)));
    if (dot(uv, nn) > 0) nn = -nn;
    double eta = (k & 1) ? 1.5 : 1.0 / 1.5;
    vec3 r = refract(uv, nn, eta), rf = reflect(uv, nn);
    double cosv = std::fmin(dot(-uv, nn), 1.0);
    pvec(uv); pvec(nn); p17(eta); pvec(r); pvec(rf);
    p17(dielectric::reflectance(cosv, eta));
    std::printf("\n");
  }
  std::printf("near_zero 6\n");
  const double nz[6][3] = {{0, 0, 0}, {-1, 0, 0}, {1e-9, -1e-9, 1e-9}, {2e-8, 0, 0}, {0, 2e-8, 0}, {-5, 1e-9, 1e-9}};
  for (auto &e : nz) { vec3 v(e[0], e[1], e[2]); pvec(v); std::printf(" %d\n", v.near_zero() ? 1 : 0); }
  // scatter (material.h) with srand(k): lambertian / metal / dielectric.
  std::printf("scatter %d\n", n);
  for (int k = 0; k < n; k++) {
    int kind = k % 3;
    shared_ptr<material> m;
    if (kind == 0) m = make_shared<lambertian>(color(g.uni(), g.uni(), g.uni()));
    else if (kind == 1) m = make_shared<metal>(color(g.range(0.5, 1), g.range(0.5, 1), g.range(0.5, 1)), g.range(0, 1.2));
    else m = make_shared<dielectric>(1.5);
    vec3 din(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1));
    hit_record rec;
    rec.p = point3(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1));
    vec3 outward = unit_vector(vec3(g.range(-1, 1), g.range(-1, 1), g.range(-1, 1)));
    rec.set_face_nromal(ray(point3(0, 0, 0), din), outward);
    rec.t = 1.0;
    rec.mat_ptr = m;
    srand(static_cast<unsigned>(1000 + k));
    color att(0, 0, 0);
    ray sc;
    bool ok = m->scatter(ray(point3(0, 0, 0), din), rec, att, sc);
    int next = rand();
    int mk; double mp[4];
    material_row(m, &mk, mp);
    std::printf("%d", mk); p17(mp[0]); p17(mp[1]); p17(mp[2]); p17(mp[3]);
    pvec(din); pvec(rec.p); pvec(rec.normal); std::printf(" %d", rec.front_face ? 1 : 0);
    std::printf(" %d", ok ? 1 : 0); pvec(att); pvec(sc.origin()); pvec(sc.direction());
    std::printf(" %d %d\n", k, next);
  }
}

// The reference's multi-threaded pixel loop (main.cpp:313-338) on `threads`
// std::threads over contiguous batches, timed by wall clock (the reference
// times with clock(), which is CPU time summed over threads: main.cpp:323-342).
void bench(int threads, int W, int H, int spp, int depth) {
  hittable_list world = random_scene();
  camera cam = final_camera(double(W) / double(H));
  const int size = W * H;
  std::vector<shared_ptr<color>> img(size);
  const int batch = static_cast<int>(std::ceil(size / double(threads)));
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  for (int i = 0; i < threads; i++) {
    int start = batch * i, end = std::min(batch * (i + 1), size);
    if (start >= end) break;
    ts.emplace_back(worker, start, end, std::ref(img), W, H, world, cam, spp, depth);
  }
  for (auto &t : ts) t.join();
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  double checksum = 0;
  for (int p = 0; p < size; p++) checksum += img[p]->x() + img[p]->y() + img[p]->z();
  std::printf("{\"threads\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"depth\": %d, "
              "\"seconds\": %.6f, \"msamples_per_s\": %.6f, \"checksum\": %.9g}\n",
              threads, W, H, spp, depth, sec, double(size) * spp / sec / 1e6, checksum / (double(size) * spp));
}

}  // namespace

int main(int argc, char **argv) {
  std::string cmd = argc > 1 ? argv[1] : "";
  if (cmd == "scene") {
    dump_world(random_scene());
  } else if (cmd == "learn_scene") {
    dump_world(learn_world());
  } else if (cmd == "camera" && argc > 2) {
    dump_camera(is_final(argv[2]) ? final_camera(3.0 / 2.0) : learn_camera(16.0 / 9.0));
  } else if (cmd == "kats" && argc > 3) {
    kats(argv[2], std::atoi(argv[3]));
  } else if (cmd == "image" && argc > 7) {
    image(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]), argv[7]);
  } else if (cmd == "funcs" && argc > 2) {
    funcs(std::atoi(argv[2]));
  } else if (cmd == "bench" && argc > 6) {
    bench(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]));
  } else {
    std::fprintf(stderr,
                 "usage: %s scene | learn_scene | camera final|learn | kats final|learn N |\n"
                 "       image final|learn W H SPP DEPTH OUT.f64 | funcs N | bench THREADS W H SPP DEPTH\n",
                 argv[0]);
    return 2;
  }
  return 0;
}
