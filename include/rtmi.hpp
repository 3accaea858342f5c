// include/rtmi.hpp — header-only C++ drop-in adapter for rt_in_one_weekend/.
//
// Include AFTER the reference's headers (camera.h, hittable_list.h, sphere.h,
// material.h): it walks the reference's own types and forwards them through
// the C ABI of librtmi.so (include/rtmi.h).  Replacing the 16-thread pixel
// loop of parallel_render() (rt_in_one_weekend/main.cpp:313-338) is then
//
//     std::vector<shared_ptr<color>> img(size);
//     int rc = rtmi::render(image_width, image_height, samples_per_pixel,
//                           max_depth, world, cam, img);
//
// after which the reference's unchanged output loop (main.cpp:344-355) writes
// the PPM.  img is filled exactly as worker() fills it (main.cpp:284-285):
// per-pixel colour SUMS, index j*W + i, row 0 = bottom.  See INTEGRATION.md.
#ifndef RTMI_HPP
#define RTMI_HPP

#include <cstdint>
#include <memory>
#include <vector>

#include "rtmi.h"

namespace rtmi {

// hittable_list::objects (hittable_list.h:16-17) as rt_scene arrays.
struct FlatScene {
  std::vector<double> center_radius, mat_params;
  std::vector<int32_t> mat_kind;
  rt_scene view() const {
    return rt_scene{static_cast<int32_t>(mat_kind.size()), center_radius.data(), mat_kind.data(), mat_params.data()};
  }
};

// sphere (sphere.h:7-19) with lambertian / metal / dielectric (material.h)
// -> flat arrays.  Any other hittable or material -> RT_EUNSUPPORTED.
inline int flatten(const hittable_list &world, FlatScene &out) {
  out = FlatScene{};
  for (const auto &obj : world.objects) {
    auto s = std::dynamic_pointer_cast<sphere>(obj);
    if (!s) return RT_EUNSUPPORTED;
    double p[4] = {0, 0, 0, 0};
    int32_t kind;
    if (auto l = std::dynamic_pointer_cast<lambertian>(s->mat_ptr)) {
      kind = RT_MAT_LAMBERTIAN;
      p[0] = l->albedo.x(); p[1] = l->albedo.y(); p[2] = l->albedo.z();
    } else if (auto m = std::dynamic_pointer_cast<metal>(s->mat_ptr)) {
      kind = RT_MAT_METAL;
      p[0] = m->albedo.x(); p[1] = m->albedo.y(); p[2] = m->albedo.z(); p[3] = m->fuzz;
    } else if (auto d = std::dynamic_pointer_cast<dielectric>(s->mat_ptr)) {
      kind = RT_MAT_DIELECTRIC;
      p[3] = d->ir;
    } else {
      return RT_EUNSUPPORTED;
    }
    out.center_radius.insert(out.center_radius.end(), {s->center.x(), s->center.y(), s->center.z(), s->radius});
    out.mat_params.insert(out.mat_params.end(), p, p + 4);
    out.mat_kind.push_back(kind);
  }
  return RT_OK;
}

// camera public fields (camera.h:64-70) -> rt_camera.
inline rt_camera to_camera(const camera &c) {
  rt_camera r;
  auto put = [](double *dst, const vec3 &v) { dst[0] = v.x(); dst[1] = v.y(); dst[2] = v.z(); };
  put(r.origin, c.origin);
  put(r.lower_left_corner, c.lower_left_corner);
  put(r.horizontal, c.horizontal);
  put(r.vertical, c.vertical);
  put(r.u, c.u);
  put(r.v, c.v);
  put(r.w, c.w);
  r.lens_radius = c.lens_radius;
  return r;
}

// Render every pixel of the image on the GPU(s) into the sums the reference's
// output loop expects.  n_gpus = 1: one device (rt_render); n_gpus != 1:
// interleaved rows over the devices + one RCCL gather (rt_render_multi,
// 0 = all visible).  Returns RT_OK or a negative RT_E* code (rt_last_error()).
template <class Color>
int render(int image_width, int image_height, int samples_per_pixel, int max_depth, const hittable_list &world,
           const camera &cam, std::vector<std::shared_ptr<Color>> &img, uint64_t seed = 1984, int n_gpus = 1,
           int device = 0) {
  FlatScene fs;
  int rc = flatten(world, fs);
  if (rc != RT_OK) return rc;
  const rt_scene sc = fs.view();
  const rt_camera rc_cam = to_camera(cam);
  const size_t size = static_cast<size_t>(image_width) * image_height;
  std::vector<float> sum(size * 3);
  if (n_gpus == 1) {
    rt_ctx *ctx = nullptr;
    if ((rc = rt_ctx_create(device, &ctx)) != RT_OK) return rc;
    rc = rt_ctx_set_scene(ctx, &sc);
    if (rc == RT_OK) rc = rt_render(ctx, &rc_cam, image_width, image_height, samples_per_pixel, max_depth, seed, sum.data());
    rt_ctx_destroy(ctx);
  } else {
    rc = rt_render_multi(&sc, &rc_cam, image_width, image_height, samples_per_pixel, max_depth, seed, n_gpus, sum.data());
  }
  if (rc != RT_OK) return rc;
  img.resize(size);
  for (size_t p = 0; p < size; p++) img[p] = std::make_shared<Color>(sum[3 * p], sum[3 * p + 1], sum[3 * p + 2]);
  return RT_OK;
}

}  // namespace rtmi

#endif  // RTMI_HPP
