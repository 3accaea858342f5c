// rtmi_nw_types.h — flattened Next-Week scene records, shared by the host
// scene builder (rtmi_nw_scene.cpp) and the gfx950 kernels (rtmi_nw.hip).
// Layout and semantics: DESIGN.md §9.  Not installed.
#pragma once

#include <cstdint>

namespace rtmi {
namespace nw {

// object kinds (the leaf hittables of rt_next_week/cuda/)
enum ObjKind : int32_t {
  kSphere = 0,        // sphere.h            g0 = {c, r}
  kMovingSphere = 1,  // moving_sphere.h     g0 = {c0, r}, g1 = {c1, time0}, g2.x = time1
  kRectXY = 2,        // aarect.h xy_rect    g0 = {x0, x1, y0, y1}, g1.x = k
  kRectXZ = 3,        //          xz_rect    g0 = {x0, x1, z0, z1}, g1.x = k
  kRectYZ = 4,        //          yz_rect    g0 = {y0, y1, z0, z1}, g1.x = k
  kBox = 5,           // box.h               g0 = {p0, 0}, g1 = {p1, 0}
  kMedium = 6,        // constant_medium.h   boundary geometry as its kind (aux & 255), g2.w = -1/density,
                      //                     aux >> 8 = scattering-distance samples
};

// material kinds = RT_NW_* (rtmi_nw.h)
enum MatKind : int32_t { kLambertian = 0, kMetal = 1, kDielectric = 2, kDiffuseLight = 3, kIsotropic = 4 };
// texture kinds
enum TexKind : int32_t { kSolid = 0, kChecker = 1, kNoise = 2, kImage = 3 };

struct Obj {  // 64 B
  float g0[4], g1[4], g2[4];
  int32_t kind, mat, inst, aux;  // aux: medium -> boundary kind | samples << 8; other objects -> twin
                                 // medium + 1 (0: none): the medium whose boundary this object is
};
constexpr int kMaxMedia = 32;
// The device's record of a non-medium object (48 B: three float4 loads, 25%
// less LDS than Obj): media live in their own list, so only the moving
// sphere's time1 remains of g2.
struct DevObj {
  float g0[4], g1[4];
  int32_t ka;  // kind | aux << 8 (one 32-bit field: no sub-dword loads)
  int32_t mat;
  float t1;  // moving sphere: time1 (Obj g2[0])
  int32_t inst;
};
static_assert(sizeof(DevObj) == 48, "DevObj layout");
struct Inst {  // 32 B; world = translate(rotate_y(local)) (hittable.h:49-189)
  float c, s;      // cos, sin of the composed rotate_y angle
  float off[3];    // composed translation
  int32_t flags;   // bit 0 rotation present, bit 1 translation present
  int32_t pad[2];
};
struct Mat {  // 16 B
  int32_t kind, tex;
  float fuzz, ir;
};
struct Tex {  // 32 B
  int32_t kind, a, b, pad;  // checker: a = even, b = odd; noise: a = perlin; image: a = image
  float rgb[3], scale;
};
struct Image {
  int32_t offset, w, h, pad;  // offset into the image byte pool; w = 0: no data (cyan)
};

constexpr int kPerlinN = 256;
constexpr int kNodeLeafMax = 4;

static_assert(sizeof(Obj) == 64, "Obj layout");
static_assert(sizeof(Inst) == 32, "Inst layout");

}  // namespace nw
}  // namespace rtmi
