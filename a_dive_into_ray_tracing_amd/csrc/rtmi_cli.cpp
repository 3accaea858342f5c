// rtmi_cli.cpp — rtmi_render, the host driver: rt_in_one_weekend/main.cpp's
// parallel_render() (main.cpp:292-360) and learn() (main.cpp:184-263) with
// the pixel loop replaced by librtmi (C ABI only).  Defaults reproduce the
// reference's constants: final scene, 1200x800 (3:2), 500 spp, depth 50.
//
//   rtmi_render [--scene final|learn] [--width W] [--height H] [--spp S]
//               [--depth D] [--seed N] [--gpus G] [--out FILE|-] [--p6]
//               [--tile-w 8|16|32|64] [--chunk N]
//
// --gpus 1 uses rt_render on device 0; --gpus G>1 (or 0 = all) uses
// rt_render_multi (interleaved rows + one RCCL gather).  Timing goes to
// stderr as one JSON line (wall clock, unlike the reference's clock(), which
// sums CPU time over threads: main.cpp:323-342).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtmi.h"

static int die(const char *what, int rc) {
  std::fprintf(stderr, "rtmi_render: %s failed (%d): %s\n", what, rc, rt_last_error());
  return 1;
}

int main(int argc, char **argv) {
  std::string scene = "final", out = "-";
  int W = 1200, H = -1, spp = 500, depth = 50, gpus = 1, p6 = 0, tile_w = 8, chunk = 0;
  unsigned long long seed = 1984;
  for (int a = 1; a < argc; a++) {
    auto need = [&](const char *f) -> const char * {
      if (a + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", f); std::exit(2); }
      return argv[++a];
    };
    if (!std::strcmp(argv[a], "--scene")) scene = need("--scene");
    else if (!std::strcmp(argv[a], "--width")) W = std::atoi(need("--width"));
    else if (!std::strcmp(argv[a], "--height")) H = std::atoi(need("--height"));
    else if (!std::strcmp(argv[a], "--spp")) spp = std::atoi(need("--spp"));
    else if (!std::strcmp(argv[a], "--depth")) depth = std::atoi(need("--depth"));
    else if (!std::strcmp(argv[a], "--seed")) seed = std::strtoull(need("--seed"), nullptr, 10);
    else if (!std::strcmp(argv[a], "--gpus")) gpus = std::atoi(need("--gpus"));
    else if (!std::strcmp(argv[a], "--out")) out = need("--out");
    else if (!std::strcmp(argv[a], "--tile-w")) tile_w = std::atoi(need("--tile-w"));
    else if (!std::strcmp(argv[a], "--chunk")) chunk = std::atoi(need("--chunk"));
    else if (!std::strcmp(argv[a], "--p6")) p6 = 1;
    else {
      std::fprintf(stderr, "usage: %s [--scene final|learn] [--width W] [--height H] [--spp S] [--depth D]\n"
                           "          [--seed N] [--gpus G] [--out FILE|-] [--p6] [--tile-w T] [--chunk N]\n", argv[0]);
      return 2;
    }
  }
  const bool learn = scene == "learn";
  if (!learn && scene != "final") { std::fprintf(stderr, "unknown scene %s\n", scene.c_str()); return 2; }
  const double aspect = learn ? 16.0 / 9.0 : 3.0 / 2.0;          // main.cpp:186 / :294
  if (learn && W == 1200) W = 800;                                // main.cpp:187
  if (H < 0) H = static_cast<int>(W / aspect);                    // main.cpp:188 / :296
  if (learn && spp == 500) spp = 100;                             // main.cpp:189

  std::vector<double> geom(4 * 600), mat(4 * 600);
  std::vector<int32_t> kind(600);
  int32_t n = 0;
  int rc = learn ? rt_scene_learn(geom.data(), kind.data(), mat.data(), 600, &n)
                 : rt_scene_random(1, geom.data(), kind.data(), mat.data(), 600, &n);
  if (rc) return die("scene", rc);
  rt_scene sc{n, geom.data(), kind.data(), mat.data()};

  rt_camera cam;
  const double vup[3] = {0, 1, 0};
  if (learn) {
    const double lf[3] = {3, 3, 2}, la[3] = {0, 0, -1};         // main.cpp:212-216
    const double d[3] = {lf[0] - la[0], lf[1] - la[1], lf[2] - la[2]};
    rc = rt_camera_init(&cam, lf, la, vup, 20, double(W) / H, 0.5, std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]));
  } else {
    const double lf[3] = {13, 2, 3}, la[3] = {0, 0, 0};         // main.cpp:304-311
    rc = rt_camera_init(&cam, lf, la, vup, 20, double(W) / H, 0.1, 10.0);
  }
  if (rc) return die("camera", rc);

  std::vector<float> sum(size_t(W) * H * 3);
  double seconds = 0;
  if (gpus == 1) {
    rt_ctx *ctx = nullptr;
    if ((rc = rt_ctx_create(0, &ctx))) return die("rt_ctx_create", rc);
    if ((rc = rt_ctx_set_scene(ctx, &sc))) return die("rt_ctx_set_scene", rc);
    if ((rc = rt_ctx_set_tuning(ctx, tile_w, chunk))) return die("rt_ctx_set_tuning", rc);
    auto t0 = std::chrono::steady_clock::now();
    if ((rc = rt_render(ctx, &cam, W, H, spp, depth, seed, sum.data()))) return die("rt_render", rc);
    seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    rt_ctx_destroy(ctx);
  } else {
    auto t0 = std::chrono::steady_clock::now();
    if ((rc = rt_render_multi(&sc, &cam, W, H, spp, depth, seed, gpus, sum.data()))) return die("rt_render_multi", rc);
    seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  std::fprintf(stderr,
               "{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"depth\": %d, \"gpus\": %d, "
               "\"seconds\": %.6f, \"msamples_per_s\": %.3f}\n",
               scene.c_str(), W, H, spp, depth, gpus, seconds, double(W) * H * spp / seconds / 1e6);
  if ((rc = rt_write_ppm(out.c_str(), sum.data(), W, H, spp, p6))) return die("rt_write_ppm", rc);
  return 0;
}
