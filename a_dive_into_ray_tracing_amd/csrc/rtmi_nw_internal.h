// rtmi_nw_internal.h — host-side interface between the Next-Week scene
// builder (rtmi_nw_scene.cpp) and the device half (rtmi_nw.hip).  Not installed.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rtmi_nw.h"
#include "rtmi_nw_types.h"

namespace rtmi {
namespace nw {

// BVH node over objects: DFS order with skip links (the RTIOW BVH's format,
// rtmi_path.h BvhNode): leaf = first << 4 | count, -1 for inner nodes.
struct Node {
  float bmin[3];
  int32_t skip;
  float bmax[3];
  int32_t leaf;
};

// What the device renders: flattened records in BVH leaf order, plus each
// object's world-insertion index (the tie-break key).
struct DeviceScene {
  std::vector<Obj> obj;          // non-media objects, BVH leaf order; aux = twin medium's index in med + 1
  std::vector<int32_t> obj_id;   // insertion index of obj[k]
  std::vector<Obj> med;          // media, insertion order
  std::vector<int32_t> med_id;   // their insertion indices
  std::vector<Inst> inst;
  std::vector<Mat> mat;
  std::vector<Tex> tex;
  std::vector<float> perlin_vec;     // n_perlin * 256 * 4
  std::vector<int32_t> perlin_perm;  // n_perlin * 768
  std::vector<uint8_t> image_px;
  std::vector<Image> image;
  std::vector<Node> nodes;
  float background[3];
  bool has_media;
  // uniform grid over the same objects; grid_ok false when
  // the scene has none (no small objects, or it would not fit in LDS)
  bool grid_ok = false;
  float grid_g0[3], grid_h[3], grid_inv_h[3], grid_g1[3];
  int32_t grid_n[3];
  int32_t grid_max_cell = 0;               // largest cell's object count
  std::vector<uint16_t> grid_cell_start;   // ncells + 1
  std::vector<uint16_t> grid_refs;         // object indices (leaf order) per cell
  std::vector<int32_t> grid_big;           // objects tested brute force beside the grid (leaf order)
};

// Flatten the world and build the BVH (RT_OK or RT_E*).
int build_device_scene(rt_nw_scene *s, DeviceScene &out);
// rt_nw_scene_grid_stats: the grid of build_device_scene, host only.
int scene_grid_stats(rt_nw_scene *s, int32_t *dims3, int32_t *max_cell, int32_t *n_big, int32_t *n_refs);

}  // namespace nw
}  // namespace rtmi
