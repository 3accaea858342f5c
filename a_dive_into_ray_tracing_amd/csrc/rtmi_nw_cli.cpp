// rtmi_nw_cli.cpp — rtmi_nw_render, the Next-Week host driver: the reference's
// rt_next_week/cuda/main.cu main() (main.cu:492-600) with create_world's
// scene switch as a flag and the render on librtmi (C ABI only).  Defaults
// are the reference's constants: scene 8 (the final scene, `switch (0)` falls
// to `default: case 8`), 800x800, 5000 spp, depth 50.
//
//   rtmi_nw_render [--scene 1..8|final|cornell_box|...] [--width W] [--height H]
//                  [--spp S] [--depth D] [--seed N] [--texture FILE.ppm]
//                  [--out FILE|-] [--p6] [--rtl]
//
// --texture is the earth image as a binary PPM (P6; the reference decodes
// earthmap.jpeg with stb_image, main.cu:497-510 — convert it once, e.g. with
// PIL).  The P3 output follows main.cu:563-575: int(255.99 * sqrt(mean)) per
// channel, top row first, NOT clamped (lights print values above 255, as the
// reference does); --p6 clamps to bytes.  Timing goes to stderr as JSON.
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtmi_nw.h"

static int die(const char *what, int rc) {
  std::fprintf(stderr, "rtmi_nw_render: %s failed (%d): %s\n", what, rc, rt_last_error());
  return 1;
}

// binary PPM (P6, maxval 255) -> rgb bytes, row 0 at the top
static bool read_p6(const char *path, std::vector<uint8_t> &px, int &w, int &h) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  char magic[3] = {0};
  int maxv = 0;
  bool ok = std::fscanf(f, "%2s", magic) == 1 && !std::strcmp(magic, "P6");
  auto skip = [&] {  // whitespace and '#' comments between header fields
    int c;
    while ((c = std::fgetc(f)) != EOF) {
      if (c == '#') {
        while ((c = std::fgetc(f)) != EOF && c != '\n') {}
      } else if (!std::isspace(c)) {
        std::ungetc(c, f);
        return;
      }
    }
  };
  if (ok) { skip(); ok = std::fscanf(f, "%d", &w) == 1; }
  if (ok) { skip(); ok = std::fscanf(f, "%d", &h) == 1; }
  if (ok) { skip(); ok = std::fscanf(f, "%d", &maxv) == 1 && maxv == 255 && w > 0 && h > 0 && w <= 65536 && h <= 65536; }
  if (ok) ok = std::fgetc(f) != EOF;  // the single whitespace byte before the raster
  if (ok) {
    px.resize(size_t(w) * h * 3);
    ok = std::fread(px.data(), 1, px.size(), f) == px.size();
  }
  std::fclose(f);
  return ok;
}

int main(int argc, char **argv) {
  std::string scene = "8", out = "-", texture;
  int W = 800, H = -1, spp = 5000, depth = 50, p6 = 0, rtl = 0;
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
    else if (!std::strcmp(argv[a], "--texture")) texture = need("--texture");
    else if (!std::strcmp(argv[a], "--out")) out = need("--out");
    else if (!std::strcmp(argv[a], "--p6")) p6 = 1;
    else if (!std::strcmp(argv[a], "--rtl")) rtl = 1;
    else {
      std::fprintf(stderr, "usage: %s [--scene 1..8|name] [--width W] [--height H] [--spp S] [--depth D]\n"
                           "          [--seed N] [--texture FILE.ppm] [--out FILE|-] [--p6] [--rtl]\n", argv[0]);
      return 2;
    }
  }
  static const char *names[] = {"", "random", "two_spheres", "two_perlin_spheres", "earth", "simple_light",
                                "cornell_box", "cornell_smoke", "final"};
  int which = std::atoi(scene.c_str());
  for (int k = 1; k <= 8; ++k)
    if (scene == names[k]) which = k;
  if (which < 1 || which > 8) { std::fprintf(stderr, "unknown scene %s\n", scene.c_str()); return 2; }
  if (H < 0) H = W;  // aspect_ratio = 1.0, main.cu:517-519
  std::vector<uint8_t> img;
  int iw = 0, ih = 0;
  if (!texture.empty() && !read_p6(texture.c_str(), img, iw, ih)) {
    std::fprintf(stderr, "cannot read P6 texture %s\n", texture.c_str());
    return 2;
  }

  rt_nw_scene *s = nullptr;
  rt_nw_camera cam;
  int rc;
  if ((rc = rt_nw_scene_create(&s))) return die("rt_nw_scene_create", rc);
  if ((rc = rt_nw_scene_preset(s, which, img.empty() ? nullptr : img.data(), iw, ih, double(W) / H,
                               rtl ? RT_NW_ARGS_RTL : 0, &cam)))
    return die("rt_nw_scene_preset", rc);
  rt_nw_ctx *ctx = nullptr;
  if ((rc = rt_nw_ctx_create(0, &ctx))) return die("rt_nw_ctx_create", rc);
  if ((rc = rt_nw_ctx_set_scene(ctx, s))) return die("rt_nw_ctx_set_scene", rc);
  std::vector<float> sum(size_t(W) * H * 3);
  const auto t0 = std::chrono::steady_clock::now();
  if ((rc = rt_nw_render(ctx, &cam, W, H, spp, depth, seed, sum.data()))) return die("rt_nw_render", rc);
  const double seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t segs = 0;
  rt_nw_ctx_last_segments(ctx, &segs);
  std::fprintf(stderr,
               "{\"scene\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"depth\": %d, \"seconds\": %.6f, "
               "\"msamples_per_s\": %.3f, \"segments_per_sample\": %.4f}\n",
               which, W, H, spp, depth, seconds, double(W) * H * spp / seconds / 1e6, double(segs) / (double(W) * H * spp));
  rt_nw_ctx_destroy(ctx);
  rt_nw_scene_destroy(s);

  FILE *f = out == "-" ? stdout : std::fopen(out.c_str(), "wb");
  if (!f) { std::fprintf(stderr, "cannot open %s\n", out.c_str()); return 1; }
  std::fprintf(f, p6 ? "P6\n%d %d\n255\n" : "P3\n%d %d\n255\n", W, H);
  for (int j = H - 1; j >= 0; j--)  // main.cu:567-575
    for (int i = 0; i < W; i++) {
      int v[3];
      for (int c = 0; c < 3; c++) {
        const float mean = sum[(size_t(j) * W + i) * 3 + c] / float(spp);
        v[c] = int(255.99 * double(std::sqrt(mean)));
      }
      if (p6) {
        for (int c = 0; c < 3; c++) std::fputc(v[c] < 0 ? 0 : v[c] > 255 ? 255 : v[c], f);
      } else {
        std::fprintf(f, "%d %d %d\n", v[0], v[1], v[2]);
      }
    }
  if (f != stdout) std::fclose(f);
  return 0;
}
