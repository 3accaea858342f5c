// rtmi_cli.cpp — rtmi_render, the host driver: rt_in_one_weekend/main.cpp's
// parallel_render() (main.cpp:292-360) and learn() (main.cpp:184-263) with
// the pixel loop replaced by librtmi (C ABI only).  Defaults reproduce the
// reference's constants: final scene, 1200x800 (3:2), 500 spp, depth 50.
//
//   rtmi_render [--scene final|learn] [--width W] [--height H] [--spp S]
//               [--depth D] [--seed N] [--gpus G] [--out FILE|-] [--p6]
//               [--tile-w 0|8|16|32|64] [--chunk N] [--scene-file F]
//               [--save-scene F] [--pfm F] [--pass-spp N [--checkpoint F]]
//               [--accel grid|bvh|none]
//
// --gpus 1 uses rt_render on device 0; --gpus G>1 (or 0 = all) uses
// rt_render_multi (interleaved rows + one RCCL gather).  --pass-spp renders
// progressively on device 0 (rt_render_pass, bounded kernels) and, with
// --checkpoint, saves the accumulator after every pass and resumes from it
// (SURVEY §8(f) rank 2).  --scene-file reads a scene text file instead of
// generating one (rt_scene_read), --save-scene writes the scene used,
// --pfm writes the pre-gamma mean as PFM next to the PPM.  Timing goes to
// stderr as one JSON line (wall clock, unlike the reference's clock(), which
// sums CPU time over threads: main.cpp:323-342).
#include <algorithm>
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
  std::string scene = "final", out = "-", scene_file, save_scene, pfm, checkpoint;
  int W = 1200, H = -1, spp = 500, depth = 50, gpus = 1, p6 = 0, tile_w = 0, chunk = 0, pass_spp = 0;
  int accel = RT_ACCEL_GRID;  // closest-hit structure (same image for every choice)
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
    else if (!std::strcmp(argv[a], "--scene-file")) scene_file = need("--scene-file");
    else if (!std::strcmp(argv[a], "--save-scene")) save_scene = need("--save-scene");
    else if (!std::strcmp(argv[a], "--pfm")) pfm = need("--pfm");
    else if (!std::strcmp(argv[a], "--pass-spp")) pass_spp = std::atoi(need("--pass-spp"));
    else if (!std::strcmp(argv[a], "--checkpoint")) checkpoint = need("--checkpoint");
    else if (!std::strcmp(argv[a], "--accel")) {
      const std::string v = need("--accel");
      accel = v == "grid" ? RT_ACCEL_GRID : v == "bvh" ? RT_ACCEL_BVH : v == "none" ? RT_ACCEL_NONE : -1;
      if (accel < 0) { std::fprintf(stderr, "unknown --accel %s\n", v.c_str()); return 2; }
    }
    else {
      std::fprintf(stderr, "usage: %s [--scene final|learn] [--width W] [--height H] [--spp S] [--depth D]\n"
                           "          [--seed N] [--gpus G] [--out FILE|-] [--p6] [--tile-w T] [--chunk N]\n"
                           "          [--scene-file F] [--save-scene F] [--pfm F] [--pass-spp N [--checkpoint F]]\n"
                           "          [--accel grid|bvh|none]\n",
                   argv[0]);
      return 2;
    }
  }
  const bool learn = scene == "learn";
  if (!learn && scene != "final") { std::fprintf(stderr, "unknown scene %s\n", scene.c_str()); return 2; }
  const double aspect = learn ? 16.0 / 9.0 : 3.0 / 2.0;          // main.cpp:186 / :294
  if (learn && W == 1200) W = 800;                                // main.cpp:187
  if (H < 0) H = static_cast<int>(W / aspect);                    // main.cpp:188 / :296
  if (learn && spp == 500) spp = 100;                             // main.cpp:189

  if (!checkpoint.empty() && pass_spp <= 0) { std::fprintf(stderr, "--checkpoint needs --pass-spp\n"); return 2; }
  if (W < 2 || H < 2 || int64_t(W) * H > (int64_t(1) << 31) || spp < 1 || depth < 0 || gpus < 0 || pass_spp < 0) {
    std::fprintf(stderr, "rtmi_render: bad size (W, H >= 2, W*H <= 2^31, spp >= 1, depth >= 0, gpus >= 0)\n");
    return 2;
  }
  int32_t n = 0;
  int rc = 0;
  if (!scene_file.empty() && (rc = rt_scene_read(scene_file.c_str(), nullptr, nullptr, nullptr, 0, &n)) && n == 0)
    return die("rt_scene_read", rc);
  const int32_t cap = scene_file.empty() ? 600 : n;
  std::vector<double> geom(4 * size_t(cap)), mat(4 * size_t(cap));
  std::vector<int32_t> kind(cap);
  if (!scene_file.empty()) rc = rt_scene_read(scene_file.c_str(), geom.data(), kind.data(), mat.data(), cap, &n);
  else if (learn) rc = rt_scene_learn(geom.data(), kind.data(), mat.data(), cap, &n);
  else rc = rt_scene_random(1, geom.data(), kind.data(), mat.data(), cap, &n);
  if (rc) return die("scene", rc);
  rt_scene sc{n, geom.data(), kind.data(), mat.data()};
  if (!save_scene.empty() && (rc = rt_scene_write(save_scene.c_str(), &sc))) return die("rt_scene_write", rc);

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
  int spp_resumed = 0;
  if (pass_spp > 0) {
    rt_ctx *ctx = nullptr;
    if ((rc = rt_ctx_create(0, &ctx))) return die("rt_ctx_create", rc);
    if ((rc = rt_ctx_set_scene(ctx, &sc))) return die("rt_ctx_set_scene", rc);
    if ((rc = rt_ctx_set_tuning(ctx, tile_w, chunk))) return die("rt_ctx_set_tuning", rc);
    if ((rc = rt_ctx_set_accel(ctx, accel))) return die("rt_ctx_set_accel", rc);
    if ((rc = rt_accum_reset(ctx, W, H))) return die("rt_accum_reset", rc);
    int done = 0;
    if (!checkpoint.empty()) {
      if (FILE *probe = std::fopen(checkpoint.c_str(), "rb")) {
        std::fclose(probe);
        if ((rc = rt_accum_load(ctx, checkpoint.c_str(), &sc, &cam, W, H, 0, 1, H, depth, seed, &done)))
          return die("rt_accum_load", rc);
        spp_resumed = done;
      }
    }
    auto t0 = std::chrono::steady_clock::now();
    while (done < spp) {
      const int k = std::min(pass_spp, spp - done);
      if ((rc = rt_render_pass(ctx, &cam, W, H, done, k, depth, seed, 0, 1, H, nullptr))) return die("rt_render_pass", rc);
      done += k;
      if (!checkpoint.empty() && (rc = rt_accum_save(ctx, checkpoint.c_str(), &sc, &cam, H, 0, 1, depth, seed)))
        return die("rt_accum_save", rc);
      if ((rc = rt_ctx_synchronize(ctx))) return die("rt_ctx_synchronize", rc);
      std::fprintf(stderr, "{\"pass_done_spp\": %d}\n", done);
    }
    if ((rc = rt_accum_resolve(ctx, nullptr, sum.data(), nullptr))) return die("rt_accum_resolve", rc);
    seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    rt_ctx_destroy(ctx);
  } else if (gpus == 1) {
    rt_ctx *ctx = nullptr;
    if ((rc = rt_ctx_create(0, &ctx))) return die("rt_ctx_create", rc);
    if ((rc = rt_ctx_set_scene(ctx, &sc))) return die("rt_ctx_set_scene", rc);
    if ((rc = rt_ctx_set_tuning(ctx, tile_w, chunk))) return die("rt_ctx_set_tuning", rc);
    if ((rc = rt_ctx_set_accel(ctx, accel))) return die("rt_ctx_set_accel", rc);
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
               scene.c_str(), W, H, spp, depth, gpus, seconds, double(W) * H * (spp - spp_resumed) / seconds / 1e6);
  if ((rc = rt_write_ppm(out.c_str(), sum.data(), W, H, spp, p6))) return die("rt_write_ppm", rc);
  if (!pfm.empty() && (rc = rt_write_pfm(pfm.c_str(), sum.data(), W, H, spp))) return die("rt_write_pfm", rc);
  return 0;
}
