// oracle/ref/dropin_demo.cpp — the drop-in, demonstrated on the reference
// itself (built here by oracle/Makefile into oracle/_ref/, never copied).
//
// This is rt_in_one_weekend/main.cpp's parallel_render() (main.cpp:292-360)
// with exactly one change: the 16-std::thread worker() block (main.cpp:
// 318-338) becomes rtmi::render(...) from include/rtmi.hpp.  Scene, camera,
// the img vector of shared_ptr<color> sums and the P3 output loop are the
// reference's own code.  Usage: dropin_demo [W] [spp] [gpus] > out.ppm
#include <chrono>
#include <cstdlib>
#define main ref_main
#include REF_MAIN_CPP
#undef main
#include "../../include/rtmi.hpp"

int main(int argc, char **argv) {
  const auto aspect_ratio = 3.0 / 2.0;                                  // main.cpp:294
  const int image_width = argc > 1 ? std::atoi(argv[1]) : 1200;         // main.cpp:295
  const int image_height = static_cast<int>(image_width / aspect_ratio);
  const int samples_per_pixel = argc > 2 ? std::atoi(argv[2]) : 500;    // main.cpp:297
  const int max_depth = 50;
  const int gpus = argc > 3 ? std::atoi(argv[3]) : 1;
  auto world = random_scene();                                          // main.cpp:301
  point3 lookfrom(13, 2, 3);
  point3 lookat(0, 0, 0);
  vec3 vup(0, 1, 0);
  auto dist_to_focus = 10.0;
  auto aperture = 0.1;
  camera cam(lookfrom, lookat, vup, 20, aspect_ratio, aperture, dist_to_focus);
  int size = image_height * image_width;
  std::vector<shared_ptr<color>> img(size);
  auto t0 = std::chrono::steady_clock::now();
  // ---- replaces main.cpp:318-338 -------------------------------------
  int rc = rtmi::render(image_width, image_height, samples_per_pixel, max_depth, world, cam, img, 1984, gpus);
  if (rc != RT_OK) {
    std::cerr << "rtmi::render failed (" << rc << "): " << rt_last_error() << "\n";
    return 1;
  }
  // ---------------------------------------------------------------------
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::cerr << "took " << sec << " seconds.\n";
  std::cout << "P3\n" << image_width << ' ' << image_height << "\n255\n";  // main.cpp:344-355
  for (int j = image_height - 1; j >= 0; --j)
    for (int i = 0; i < image_width; ++i) {
      color pixel_color(img[j * image_width + i].get()->x(), img[j * image_width + i].get()->y(),
                        img[j * image_width + i].get()->z());
      write_color(std::cout, pixel_color, samples_per_pixel);
    }
  return 0;
}
