// rtmi_nw_scene.cpp — host half of the Next-Week renderer: the scene builder
// (one call per reference constructor, include/rtmi_nw.h), flattening of the
// instance tree into leaf records with composed transforms, the object BVH,
// the reference's scene presets (rt_next_week/cuda/main.cu:163-413) and the
// curand XORWOW restatement they draw from.  No device code.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>
#include <vector>

#include "rtmi_internal.h"
#include "rtmi_nw_internal.h"

using namespace rtmi;
using namespace rtmi::nw;

namespace {

enum SType { kPrim = 0, kGroup = 1, kTranslate = 2, kRotate = 3, kMediumNode = 4 };

struct SNode {
  int type = kPrim;
  int32_t kind = 0, mat = -1;  // kPrim
  double g[12] = {0};          // kPrim geometry, double (layout of Obj g0..g2)
  std::vector<int32_t> kids;   // kGroup
  int32_t child = -1;          // kTranslate / kRotate / kMediumNode
  double off[3] = {0, 0, 0};   // kTranslate
  double angle = 0;            // kRotate (degrees)
  double density = 0;          // kMediumNode
  int32_t phase_mat = -1;      // kMediumNode: its isotropic material
  int32_t samples = 1;         // kMediumNode: scattering-distance samples (rt_nw_medium_samples)
};

// world = R(theta) * local + t, R about y: (x, z) -> (c x + s z, -s x + c z)
// (rotate_y's local-to-world map, hittable.h:128-131 / 175-179)
struct Xf {
  double theta = 0;  // degrees
  double t[3] = {0, 0, 0};
  bool rot = false, trans = false;
};

struct Bounds {
  double lo[3], hi[3];
};

// curand XORWOW (cuRAND's published device generator): curand_init(seed, 0,
// 0) state set-up and curand(), curand_uniform = x * 2^-32 + 2^-33 as one
// fused multiply-add (nvcc contracts it by default) in (0, 1].
struct Xorwow {
  uint32_t v[5], d;
  explicit Xorwow(uint64_t seed) {
    const uint32_t s0 = uint32_t(seed) ^ 0xaad26b49u;
    const uint32_t s1 = uint32_t(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    d = 6615241u + t1 + t0;
    v[0] = 123456789u + t0;
    v[1] = 362436069u ^ t0;
    v[2] = 521288629u + t1;
    v[3] = 88675123u ^ t1;
    v[4] = 5783321u + t0;
  }
  uint32_t next() {
    const uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1];
    v[1] = v[2];
    v[2] = v[3];
    v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
    d += 362437u;
    return v[4] + d;
  }
  float uniform() {
    const float inv = 2.3283064e-10f;
    return std::fmaf(float(next()), inv, inv * 0.5f);
  }
  // random_float(min, max) rtweekend.h:45-48 (contracted)
  float range(float lo, float hi) { return std::fmaf(uniform(), hi - lo, lo); }
  // random_int(n) rtweekend.h:36-40: (float)n - 0.000001 in double, stored to
  // float (256 - 1e-6 rounds to 256.0f); u = 1.0f would give n: clamped
  int rint(int n) {
    const float val = float(double(float(n)) - 0.000001);
    const int r = int(uniform() * val);
    return r < n ? r : n - 1;
  }
};

}  // namespace

struct rt_nw_scene {
  std::vector<Tex> tex;
  std::vector<float> perlin_vec;
  std::vector<int32_t> perlin_perm;
  std::vector<uint8_t> image_px;
  std::vector<Image> image;
  std::vector<Mat> mat;
  std::vector<SNode> nodes;
  std::vector<int32_t> world;
  float background[3] = {0.f, 0.f, 0.f};
  // flattened view (rt_nw_scene_flat), insertion order
  bool flat_valid = false;
  std::vector<Obj> flat_obj;
  std::vector<int32_t> flat_src;  // the SNode a flattened object came from (twin detection)
  std::vector<Bounds> flat_bounds;
  std::vector<Inst> flat_inst;
};

namespace {

int add_node(rt_nw_scene *s, SNode n) {
  s->nodes.push_back(std::move(n));
  s->flat_valid = false;
  return int(s->nodes.size()) - 1;
}
bool valid_node(const rt_nw_scene *s, int32_t id) { return id >= 0 && id < int32_t(s->nodes.size()); }
bool valid_tex(const rt_nw_scene *s, int32_t id) { return id >= 0 && id < int32_t(s->tex.size()); }
bool valid_mat(const rt_nw_scene *s, int32_t id) { return id >= 0 && id < int32_t(s->mat.size()); }

int add_tex(rt_nw_scene *s, Tex t) {
  s->tex.push_back(t);
  s->flat_valid = false;
  return int(s->tex.size()) - 1;
}
int add_mat(rt_nw_scene *s, Mat m) {
  s->mat.push_back(m);
  s->flat_valid = false;
  return int(s->mat.size()) - 1;
}

Xf compose_translate(const Xf &x, const double off[3]) {
  Xf r = x;
  const double th = x.theta * M_PI / 180.0, c = std::cos(th), sn = std::sin(th);
  r.t[0] = x.t[0] + (c * off[0] + sn * off[2]);
  r.t[1] = x.t[1] + off[1];
  r.t[2] = x.t[2] + (-sn * off[0] + c * off[2]);
  r.trans = true;
  return r;
}
Xf compose_rotate(const Xf &x, double angle) {
  Xf r = x;
  r.theta = x.theta + angle;
  r.rot = true;
  return r;
}

Bounds local_bounds(const SNode &n, int32_t kind) {
  Bounds b;
  const double *g = n.g;
  auto sphere_at = [&](double cx, double cy, double cz, double r, Bounds &acc) {
    r = std::fabs(r);
    const double c[3] = {cx, cy, cz};
    for (int a = 0; a < 3; ++a) {
      acc.lo[a] = std::min(acc.lo[a], c[a] - r);
      acc.hi[a] = std::max(acc.hi[a], c[a] + r);
    }
  };
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = INFINITY;
    b.hi[a] = -INFINITY;
  }
  switch (kind) {
    case kSphere: sphere_at(g[0], g[1], g[2], g[3], b); break;
    case kMovingSphere: {
      // the centre is linear in time: its extremes over the render's times
      // (camera shutters are restricted to [0, 1]) and the sphere's own
      // interval are at the interval ends
      const double t0 = g[7], t1 = g[8];
      for (double tm : {std::min(0.0, t0), std::max(1.0, t1), t0, t1}) {
        const double f = (tm - t0) / (t1 - t0);
        sphere_at(g[0] + f * (g[4] - g[0]), g[1] + f * (g[5] - g[1]), g[2] + f * (g[6] - g[2]), g[3], b);
      }
      break;
    }
    case kRectXY: case kRectXZ: case kRectYZ: {
      const int ax_a = kind == kRectYZ ? 1 : 0;
      const int ax_b = kind == kRectXY ? 1 : 2;
      const int ax_k = kind == kRectXY ? 2 : kind == kRectXZ ? 1 : 0;
      b.lo[ax_a] = std::min(g[0], g[1]); b.hi[ax_a] = std::max(g[0], g[1]);
      b.lo[ax_b] = std::min(g[2], g[3]); b.hi[ax_b] = std::max(g[2], g[3]);
      b.lo[ax_k] = g[4]; b.hi[ax_k] = g[4];
      break;
    }
    case kBox:
      for (int a = 0; a < 3; ++a) {
        b.lo[a] = std::min(g[a], g[4 + a]);
        b.hi[a] = std::max(g[a], g[4 + a]);
      }
      break;
  }
  return b;
}

Bounds world_bounds(const Bounds &lb, const Xf &x) {
  if (!x.rot && !x.trans) return lb;
  Bounds b;
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = INFINITY;
    b.hi[a] = -INFINITY;
  }
  const double th = x.theta * M_PI / 180.0, c = std::cos(th), sn = std::sin(th);
  for (int i = 0; i < 8; ++i) {
    const double p[3] = {(i & 1) ? lb.hi[0] : lb.lo[0], (i & 2) ? lb.hi[1] : lb.lo[1], (i & 4) ? lb.hi[2] : lb.lo[2]};
    const double q[3] = {c * p[0] + sn * p[2] + x.t[0], p[1] + x.t[1], -sn * p[0] + c * p[2] + x.t[2]};
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = std::min(b.lo[a], q[a]);
      b.hi[a] = std::max(b.hi[a], q[a]);
    }
  }
  return b;
}

struct Flattener {
  rt_nw_scene *s;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, int32_t>, int32_t> inst_ids;
  int err = RT_OK;

  int32_t inst_of(const Xf &x) {
    if (!x.rot && !x.trans) return -1;
    Inst in{};
    const double th = x.theta * M_PI / 180.0;
    in.c = x.rot ? float(std::cos(th)) : 1.f;
    in.s = x.rot ? float(std::sin(th)) : 0.f;
    for (int a = 0; a < 3; ++a) in.off[a] = x.trans ? float(x.t[a]) : 0.f;
    in.flags = (x.rot ? 1 : 0) | (x.trans ? 2 : 0);
    uint32_t b[5];
    std::memcpy(&b[0], &in.c, 4);
    std::memcpy(&b[1], &in.s, 4);
    std::memcpy(&b[2], &in.off[0], 12);
    const auto key = std::make_tuple(b[0], b[1], b[2], b[3], b[4], in.flags);
    auto it = inst_ids.find(key);
    if (it != inst_ids.end()) return it->second;
    s->flat_inst.push_back(in);
    const int32_t id = int32_t(s->flat_inst.size()) - 1;
    inst_ids[key] = id;
    return id;
  }

  static void store_geom(Obj &o, const SNode &n) {
    for (int i = 0; i < 4; ++i) {
      o.g0[i] = float(n.g[i]);
      o.g1[i] = float(n.g[4 + i]);
      o.g2[i] = float(n.g[8 + i]);
    }
  }

  // the single primitive under a medium's boundary subtree
  bool boundary_prim(int32_t id, Xf x, int32_t &prim, Xf &xo) {
    const SNode &n = s->nodes[id];
    switch (n.type) {
      case kPrim: prim = id; xo = x; return true;
      case kTranslate: return boundary_prim(n.child, compose_translate(x, n.off), prim, xo);
      case kRotate: return boundary_prim(n.child, compose_rotate(x, n.angle), prim, xo);
      case kGroup:
        if (n.kids.size() == 1) return boundary_prim(n.kids[0], x, prim, xo);
        return false;
      default: return false;
    }
  }

  void emit(int32_t id, Xf x, int depth) {
    if (err) return;
    if (depth > 64) {
      err = set_error(RT_EINVAL, "rt_nw: object nesting deeper than 64 (a cycle?)");
      return;
    }
    const SNode &n = s->nodes[id];
    switch (n.type) {
      case kPrim: {
        Obj o{};
        store_geom(o, n);
        o.kind = n.kind;
        o.mat = n.mat;
        o.inst = inst_of(x);
        o.aux = 0;
        s->flat_obj.push_back(o);
        s->flat_src.push_back(id);
        s->flat_bounds.push_back(world_bounds(local_bounds(n, n.kind), x));
        return;
      }
      case kGroup:
        for (int32_t k : n.kids) emit(k, x, depth + 1);
        return;
      case kTranslate: emit(n.child, compose_translate(x, n.off), depth + 1); return;
      case kRotate: emit(n.child, compose_rotate(x, n.angle), depth + 1); return;
      case kMediumNode: {
        int32_t prim = -1;
        Xf xb;
        if (!boundary_prim(n.child, x, prim, xb)) {
          err = set_error(RT_EUNSUPPORTED, "constant_medium boundary must be one sphere, moving sphere or box");
          return;
        }
        const SNode &b = s->nodes[prim];
        if (b.kind != kSphere && b.kind != kMovingSphere && b.kind != kBox) {
          err = set_error(RT_EUNSUPPORTED, "constant_medium boundary kind %d unsupported", b.kind);
          return;
        }
        Obj o{};
        store_geom(o, b);
        o.g2[3] = float(-1.0 / n.density);  // neg_inv_density constant_medium.h:13-14
        o.kind = kMedium;
        o.aux = b.kind | (n.samples << 8);
        o.mat = n.phase_mat;
        o.inst = inst_of(xb);
        s->flat_obj.push_back(o);
        s->flat_src.push_back(prim);
        s->flat_bounds.push_back(world_bounds(local_bounds(b, b.kind), xb));
        return;
      }
    }
  }
};

int flatten(rt_nw_scene *s) {
  if (s->flat_valid) return RT_OK;
  s->flat_obj.clear();
  s->flat_src.clear();
  s->flat_bounds.clear();
  s->flat_inst.clear();
  Flattener f{s, {}, RT_OK};
  for (int32_t id : s->world) f.emit(id, Xf{}, 0);
  if (f.err) return f.err;
  // twins: an object that is also a medium's boundary (the same primitive
  // under the same transform, e.g. the final scene's glass sphere and its
  // blue interior, main.cu:386-391) is hidden where that medium hits
  int32_t n_media = 0;
  for (size_t m = 0; m < s->flat_obj.size(); ++m) {
    if (s->flat_obj[m].kind != kMedium) continue;
    ++n_media;
    for (size_t k = 0; k < s->flat_obj.size(); ++k)
      if (s->flat_obj[k].kind != kMedium && s->flat_src[k] == s->flat_src[m] && s->flat_obj[k].inst == s->flat_obj[m].inst &&
          s->flat_obj[k].aux == 0)
        s->flat_obj[k].aux = int32_t(m) + 1;
  }
  if (n_media > kMaxMedia) return set_error(RT_EUNSUPPORTED, "rt_nw: more than %d media", kMaxMedia);
  if (s->flat_obj.size() >= (size_t(1) << 27)) return set_error(RT_EINVAL, "rt_nw: too many objects");
  s->flat_valid = true;
  return RT_OK;
}

// BVH over the flattened objects, built with the surface-area heuristic
// (full sweep over the centroid order on each axis): a child's expected cost
// is its area times the summed test cost of its objects, so a huge object
// (the R=1000 ground sphere) ends up alone near the root instead of inflating
// every box on its path, as a median split leaves it.  Leaves of <=
// kNodeLeafMax objects, DFS order with skip links.  Boxes are the objects'
// double bounds, each grown by its own margin, rounded outward to float
// (the RTIOW BVH's margin argument).
struct ObjBvh {
  const std::vector<Bounds> &b;
  const std::vector<double> &w;  // per-object test cost (relative)
  const std::vector<double> &m;  // per-object box margin
  std::vector<Node> nodes;
  std::vector<int32_t> order;

  static double area(const double lo[3], const double hi[3]) {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
  void build(int32_t *ids, int cnt) {
    const int me = int(nodes.size());
    nodes.push_back(Node{});
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double glo[3] = {INFINITY, INFINITY, INFINITY}, ghi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double wsum = 0;
    for (int i = 0; i < cnt; ++i) {
      wsum += w[ids[i]];
      for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], b[ids[i]].lo[a]);
        hi[a] = std::max(hi[a], b[ids[i]].hi[a]);
        glo[a] = std::min(glo[a], b[ids[i]].lo[a] - m[ids[i]]);
        ghi[a] = std::max(ghi[a], b[ids[i]].hi[a] + m[ids[i]]);
      }
    }
    Node nd{};
    for (int a = 0; a < 3; ++a) {  // every object grown by its own margin
      nd.bmin[a] = std::nextafter(float(glo[a]), -INFINITY);
      nd.bmax[a] = std::nextafter(float(ghi[a]), INFINITY);
    }
    // best SAH split: cost = C_trav * A + A_L * W_L + A_R * W_R (A = area)
    const double pa = std::max(area(lo, hi), 1e-30);
    double best = INFINITY;
    int best_ax = -1, best_i = -1;
    std::vector<double> right_cost(cnt);
    for (int ax = 0; ax < 3 && cnt > 1; ++ax) {
      std::sort(ids, ids + cnt, [&](int32_t x, int32_t y) {
        const double cx = b[x].lo[ax] + b[x].hi[ax], cy = b[y].lo[ax] + b[y].hi[ax];
        return cx < cy || (cx == cy && x < y);
      });
      double rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY}, rw = 0;
      for (int i = cnt - 1; i > 0; --i) {  // right part = ids[i..cnt)
        rw += w[ids[i]];
        for (int a = 0; a < 3; ++a) {
          rl[a] = std::min(rl[a], b[ids[i]].lo[a]);
          rh[a] = std::max(rh[a], b[ids[i]].hi[a]);
        }
        right_cost[i] = area(rl, rh) * rw;
      }
      double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY}, lw = 0;
      for (int i = 1; i < cnt; ++i) {  // left part = ids[0..i)
        lw += w[ids[i - 1]];
        for (int a = 0; a < 3; ++a) {
          ll[a] = std::min(ll[a], b[ids[i - 1]].lo[a]);
          lh[a] = std::max(lh[a], b[ids[i - 1]].hi[a]);
        }
        const double c = area(ll, lh) * lw + right_cost[i];
        if (c < best) {
          best = c;
          best_ax = ax;
          best_i = i;
        }
      }
    }
#ifndef RTMI_NW_KTRAV
#define RTMI_NW_KTRAV 2.0
#endif
    const double kTrav = RTMI_NW_KTRAV;  // a node visit against one sphere test
    const bool leaf = cnt == 1 || (cnt <= kNodeLeafMax && pa * wsum <= kTrav * pa + best);
    if (leaf) {
      nd.leaf = (int32_t(order.size()) << 4) | cnt;
      for (int i = 0; i < cnt; ++i) order.push_back(ids[i]);
      nd.skip = me + 1;
    } else {
      std::sort(ids, ids + cnt, [&](int32_t x, int32_t y) {
        const double cx = b[x].lo[best_ax] + b[x].hi[best_ax], cy = b[y].lo[best_ax] + b[y].hi[best_ax];
        return cx < cy || (cx == cy && x < y);
      });
      build(ids, best_i);
      build(ids + best_i, cnt - best_i);
      nd.leaf = -1;
      nd.skip = int(nodes.size());
    }
    nodes[me] = nd;
  }
};

// Uniform grid over the non-media objects, the RTIOW grid's
// build (rtmi_device.hip build_grid) for general objects: an object whose box
// is more than 8x the median's largest extent (the R = 1000 ground, a
// room-sized light) is tested brute force beside the grid; the others are
// listed in every cell their margin-grown box overlaps.  Cell boundaries are
// the float values g0 + c*h the device computes (origin rounded down, size
// rounded up, so the float cells cover the box).  `order` maps leaf-order
// slots to flattened objects; refs hold leaf-order slots.
void build_obj_grid(const std::vector<Bounds> &bounds, const std::vector<double> &margin,
                    const std::vector<int32_t> &order, DeviceScene &out) {
  out.grid_ok = false;
  const int n = int(order.size());
  if (n == 0 || n > 65535) return;
  std::vector<double> ext(n);
  for (int k = 0; k < n; ++k) {
    const Bounds &b = bounds[order[k]];
    double e = 0;
    for (int a = 0; a < 3; ++a) e = std::max(e, b.hi[a] - b.lo[a]);
    ext[k] = e + 2 * margin[order[k]];
  }
  std::vector<double> sorted = ext;
  std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
  const double big_ext = 8.0 * std::max(sorted[n / 2], 1e-9);
  std::vector<int32_t> small;
  out.grid_big.clear();
  for (int k = 0; k < n; ++k) (ext[k] > big_ext ? out.grid_big : small).push_back(k);
  if (small.empty()) return;
  auto grown = [&](int k, int a, bool hi) {
    const Bounds &b = bounds[order[k]];
    return hi ? b.hi[a] + margin[order[k]] : b.lo[a] - margin[order[k]];
  };
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int32_t k : small)
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], grown(k, a, false));
      hi[a] = std::max(hi[a], grown(k, a, true));
    }
  const char *env = std::getenv("RTMI_NW_GRID_CELLS");
  // cells per object: motion-blur scene 0.25 -> 134.1 ms, 0.5 -> 118.1, 1 -> 104.6, 2 -> 113.1,
  // 4 -> 118.7 (BVH 114.0; profiles/r02/nw_grid/)
  const double per_obj = env && std::atof(env) > 0 ? std::atof(env) : 1.0;
  double e[3], vol = 1;
  for (int a = 0; a < 3; ++a) {
    e[a] = std::max(hi[a] - lo[a], 1e-6 * (1 + std::fabs(lo[a])));
    vol *= e[a];
  }
  const double cell = std::cbrt(vol / (per_obj * double(small.size())));
  int64_t total = 1;
  for (int a = 0; a < 3; ++a) {
    out.grid_n[a] = int32_t(std::min<double>(128, std::max<double>(1, std::ceil(e[a] / cell))));
    total *= out.grid_n[a];
  }
  if (total > 16384) return;
  for (int a = 0; a < 3; ++a) {
    float g0 = float(lo[a]);
    if (double(g0) > lo[a]) g0 = std::nextafter(g0, -INFINITY);
    float h = float(e[a] / out.grid_n[a]);
    while (double(g0) + double(h) * out.grid_n[a] < hi[a]) h = std::nextafter(h, INFINITY);
    out.grid_g0[a] = g0;
    out.grid_h[a] = h;
    out.grid_inv_h[a] = 1.0f / h;
    out.grid_g1[a] = std::fmaf(float(out.grid_n[a]), h, g0);
  }
  std::vector<std::vector<uint16_t>> lists(static_cast<size_t>(total));
  for (int32_t k : small) {
    int c0[3], c1[3];
    for (int a = 0; a < 3; ++a) {  // every cell [g0 + c*h, g0 + (c+1)*h] the grown box touches
      const double g0 = out.grid_g0[a], h = out.grid_h[a];
      c0[a] = std::max(0, std::min(out.grid_n[a] - 1, int(std::floor((grown(k, a, false) - g0) / h))));
      c1[a] = std::max(0, std::min(out.grid_n[a] - 1, int(std::floor((grown(k, a, true) - g0) / h))));
    }
    for (int z = c0[2]; z <= c1[2]; ++z)
      for (int y = c0[1]; y <= c1[1]; ++y)
        for (int x = c0[0]; x <= c1[0]; ++x)
          lists[size_t(x + out.grid_n[0] * (y + out.grid_n[1] * z))].push_back(uint16_t(k));
  }
  out.grid_cell_start.assign(size_t(total) + 1, 0);
  out.grid_refs.clear();
  out.grid_max_cell = 0;
  for (int64_t c = 0; c < total; ++c) {
    out.grid_cell_start[size_t(c)] = uint16_t(out.grid_refs.size());
    out.grid_refs.insert(out.grid_refs.end(), lists[size_t(c)].begin(), lists[size_t(c)].end());
    out.grid_max_cell = std::max(out.grid_max_cell, int32_t(lists[size_t(c)].size()));
    if (out.grid_refs.size() > 65535) return;
  }
  out.grid_cell_start[size_t(total)] = uint16_t(out.grid_refs.size());
  out.grid_ok = true;
}

}  // namespace

namespace rtmi {
namespace nw {

int build_device_scene(rt_nw_scene *s, DeviceScene &out) {
  if (!s) return set_error(RT_EINVAL, "null scene");
  if (int rc = flatten(s)) return rc;
  const int n_all = int(s->flat_obj.size());
  if (n_all == 0) return set_error(RT_EINVAL, "rt_nw: empty world (rt_nw_world_add)");
  // media are evaluated per segment before the BVH walk;
  // the BVH holds the other objects
  std::vector<int32_t> med_index(n_all, -1), ids;
  out.med.clear();
  out.med_id.clear();
  for (int k = 0; k < n_all; ++k) {
    if (s->flat_obj[k].kind == kMedium) {
      med_index[k] = int32_t(out.med.size());
      out.med.push_back(s->flat_obj[k]);
      out.med_id.push_back(k);
    } else {
      ids.push_back(k);
    }
  }
  double scale = 0;
  for (int32_t k : ids) {
    const Bounds &b = s->flat_bounds[k];
    for (int a = 0; a < 3; ++a) {
      if (!std::isfinite(b.lo[a]) || !std::isfinite(b.hi[a]))
        return set_error(RT_EINVAL, "rt_nw: object with non-finite bounds");
      scale = std::max(scale, std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a])));
    }
  }
  // relative test costs: a box is six rectangle tests, an instance adds a
  // ray transform
  std::vector<double> cost(n_all, 1.0);
  for (int k = 0; k < n_all; ++k) {
    const Obj &o = s->flat_obj[k];
    cost[k] = (o.kind == kBox ? 3.0 : o.kind == kMovingSphere ? 1.2 : 1.0) + (o.inst >= 0 ? 0.3 : 0.0);
  }
  // box margins (the RTIOW BVH's argument): 1e-3 of the
  // object's own coordinate scale — ~100x the float error of its hit test —
  // plus 1e-6 of the scene's, for rays from far away.  One scene-wide margin
  // of 1e-3 of the scene scale grew every small box by ~2 units next to the
  // R = 1000 ground (137 node visits per camera ray instead of ~20).
  std::vector<double> margin(n_all, 0.0);
  for (int32_t k : ids) {
    double own = 0;
    for (int a = 0; a < 3; ++a)
      own = std::max(own, std::max(std::fabs(s->flat_bounds[k].lo[a]), std::fabs(s->flat_bounds[k].hi[a])));
    margin[k] = 1e-3 * (1.0 + own) + 1e-6 * scale;
  }
  ObjBvh bvh{s->flat_bounds, cost, margin, {}, {}};
  const int n = int(ids.size());
  if (n > 0) bvh.build(ids.data(), n);
  out.nodes = std::move(bvh.nodes);
  out.obj.resize(n);
  out.obj_id.resize(n);
  for (int k = 0; k < n; ++k) {
    out.obj[k] = s->flat_obj[bvh.order[k]];
    out.obj_id[k] = bvh.order[k];
    if (out.obj[k].aux > 0) out.obj[k].aux = med_index[out.obj[k].aux - 1] + 1;  // twin -> media-list index + 1
  }
  build_obj_grid(s->flat_bounds, margin, bvh.order, out);
  out.inst = s->flat_inst;
  out.mat = s->mat;
  out.tex = s->tex;
  out.perlin_vec = s->perlin_vec;
  out.perlin_perm = s->perlin_perm;
  out.image_px = s->image_px;
  out.image = s->image;
  for (int c = 0; c < 3; ++c) out.background[c] = s->background[c];
  out.has_media = !out.med.empty();
  return RT_OK;
}

int scene_grid_stats(rt_nw_scene *s, int32_t *dims3, int32_t *max_cell, int32_t *n_big, int32_t *n_refs) {
  DeviceScene ds;
  if (int rc = build_device_scene(s, ds)) return rc;
  for (int a = 0; a < 3 && dims3; ++a) dims3[a] = ds.grid_ok ? ds.grid_n[a] : 0;
  if (max_cell) *max_cell = ds.grid_ok ? ds.grid_max_cell : 0;
  if (n_big) *n_big = ds.grid_ok ? int32_t(ds.grid_big.size()) : 0;
  if (n_refs) *n_refs = ds.grid_ok ? int32_t(ds.grid_refs.size()) : 0;
  return RT_OK;
}

}  // namespace nw
}  // namespace rtmi

// ---------------------------------------------------------------------------
// C ABI: builder
// ---------------------------------------------------------------------------
RTMI_EXPORT int rt_nw_camera_init(rt_nw_camera *cam, const double lookfrom[3], const double lookat[3],
                                  const double vup[3], double vfov_deg, double aspect_ratio, double aperture,
                                  double focus_dist, double time0, double time1) {
  if (!cam) return set_error(RT_EINVAL, "rt_nw_camera_init: null");
  if (!(time0 >= 0.0 && time1 <= 1.0 && time0 <= time1))
    return set_error(RT_EINVAL, "rt_nw_camera_init: shutter [%g, %g] must lie in [0, 1]", time0, time1);
  if (int rc = rt_camera_init(&cam->cam, lookfrom, lookat, vup, vfov_deg, aspect_ratio, aperture, focus_dist)) return rc;
  cam->time0 = time0;
  cam->time1 = time1;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_scene_create(rt_nw_scene **out) {
  if (!out) return set_error(RT_EINVAL, "null out");
  *out = new (std::nothrow) rt_nw_scene();
  return *out ? RT_OK : set_error(RT_ENOMEM, "rt_nw_scene_create");
}

RTMI_EXPORT int rt_nw_scene_destroy(rt_nw_scene *s) {
  delete s;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_tex_solid(rt_nw_scene *s, double r, double g, double b) {
  if (!s) return set_error(RT_EINVAL, "null scene");
  Tex t{};
  t.kind = kSolid;
  t.rgb[0] = float(r); t.rgb[1] = float(g); t.rgb[2] = float(b);
  return add_tex(s, t);
}

RTMI_EXPORT int rt_nw_tex_checker(rt_nw_scene *s, int32_t even, int32_t odd) {
  if (!s || !valid_tex(s, even) || !valid_tex(s, odd)) return set_error(RT_EINVAL, "rt_nw_tex_checker: bad texture");
  if (s->tex[even].kind == kChecker || s->tex[odd].kind == kChecker)
    return set_error(RT_EUNSUPPORTED, "rt_nw_tex_checker: nested checker textures");
  Tex t{};
  t.kind = kChecker;
  t.a = even;
  t.b = odd;
  return add_tex(s, t);
}

RTMI_EXPORT int rt_nw_tex_noise(rt_nw_scene *s, double scale, const float *ranvec, const int32_t *perm) {
  if (!s || !ranvec || !perm) return set_error(RT_EINVAL, "rt_nw_tex_noise: null");
  for (int i = 0; i < 3 * kPerlinN; ++i)
    if (perm[i] < 0 || perm[i] >= kPerlinN) return set_error(RT_EINVAL, "rt_nw_tex_noise: perm out of range");
  const int id = int(s->perlin_perm.size()) / (3 * kPerlinN);
  for (int i = 0; i < kPerlinN; ++i) {
    s->perlin_vec.push_back(ranvec[3 * i]);
    s->perlin_vec.push_back(ranvec[3 * i + 1]);
    s->perlin_vec.push_back(ranvec[3 * i + 2]);
    s->perlin_vec.push_back(0.f);
  }
  s->perlin_perm.insert(s->perlin_perm.end(), perm, perm + 3 * kPerlinN);
  Tex t{};
  t.kind = kNoise;
  t.a = id;
  t.scale = float(scale);
  return add_tex(s, t);
}

RTMI_EXPORT int rt_nw_tex_image(rt_nw_scene *s, const uint8_t *rgb, int32_t w, int32_t h) {
  if (!s) return set_error(RT_EINVAL, "null scene");
  Image im{};
  if (rgb) {
    if (w <= 0 || h <= 0 || int64_t(w) * h * 3 > (int64_t(1) << 30)) return set_error(RT_EINVAL, "rt_nw_tex_image: bad size");
    if (s->image_px.size() + size_t(w) * h * 3 > (size_t(1) << 31) - 1) return set_error(RT_EINVAL, "rt_nw_tex_image: pool full");
    im.offset = int32_t(s->image_px.size());
    im.w = w;
    im.h = h;
    s->image_px.insert(s->image_px.end(), rgb, rgb + size_t(w) * h * 3);
  }
  s->image.push_back(im);
  Tex t{};
  t.kind = kImage;
  t.a = int32_t(s->image.size()) - 1;
  return add_tex(s, t);
}

RTMI_EXPORT int rt_nw_mat_lambertian(rt_nw_scene *s, int32_t tex) {
  if (!s || !valid_tex(s, tex)) return set_error(RT_EINVAL, "rt_nw_mat_lambertian: bad texture");
  return add_mat(s, Mat{kLambertian, tex, 0.f, 0.f});
}
RTMI_EXPORT int rt_nw_mat_metal(rt_nw_scene *s, int32_t tex, double fuzz) {
  if (!s || !valid_tex(s, tex)) return set_error(RT_EINVAL, "rt_nw_mat_metal: bad texture");
  const float f = float(fuzz);
  return add_mat(s, Mat{kMetal, tex, f < 1.f ? f : 1.f, 0.f});  // material.h:58-62
}
RTMI_EXPORT int rt_nw_mat_dielectric(rt_nw_scene *s, double ir) {
  if (!s || !(ir > 0)) return set_error(RT_EINVAL, "rt_nw_mat_dielectric: bad argument");
  return add_mat(s, Mat{kDielectric, -1, 0.f, float(ir)});
}
RTMI_EXPORT int rt_nw_mat_diffuse_light(rt_nw_scene *s, int32_t tex) {
  if (!s || !valid_tex(s, tex)) return set_error(RT_EINVAL, "rt_nw_mat_diffuse_light: bad texture");
  return add_mat(s, Mat{kDiffuseLight, tex, 0.f, 0.f});
}
RTMI_EXPORT int rt_nw_mat_isotropic(rt_nw_scene *s, int32_t tex) {
  if (!s || !valid_tex(s, tex)) return set_error(RT_EINVAL, "rt_nw_mat_isotropic: bad texture");
  return add_mat(s, Mat{kIsotropic, tex, 0.f, 0.f});
}

RTMI_EXPORT int rt_nw_sphere(rt_nw_scene *s, const double c[3], double r, int32_t mat) {
  if (!s || !c || !valid_mat(s, mat)) return set_error(RT_EINVAL, "rt_nw_sphere: bad argument");
  if (r == 0 || !std::isfinite(r)) return set_error(RT_EINVAL, "rt_nw_sphere: radius must be finite, nonzero");
  SNode n;
  n.kind = kSphere;
  n.mat = mat;
  n.g[0] = c[0]; n.g[1] = c[1]; n.g[2] = c[2]; n.g[3] = r;
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_moving_sphere(rt_nw_scene *s, const double c0[3], const double c1[3], double t0, double t1,
                                    double r, int32_t mat) {
  if (!s || !c0 || !c1 || !valid_mat(s, mat)) return set_error(RT_EINVAL, "rt_nw_moving_sphere: bad argument");
  if (!(t1 != t0) || r == 0) return set_error(RT_EINVAL, "rt_nw_moving_sphere: time0 == time1 or zero radius");
  SNode n;
  n.kind = kMovingSphere;
  n.mat = mat;
  for (int a = 0; a < 3; ++a) {
    n.g[a] = c0[a];
    n.g[4 + a] = c1[a];
  }
  n.g[3] = r;
  n.g[7] = t0;
  n.g[8] = t1;
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_rect(rt_nw_scene *s, int32_t plane, double a0, double a1, double b0, double b1, double k,
                           int32_t mat) {
  if (!s || !valid_mat(s, mat) || plane < RT_NW_XY || plane > RT_NW_YZ) return set_error(RT_EINVAL, "rt_nw_rect: bad argument");
  SNode n;
  n.kind = kRectXY + plane;
  n.mat = mat;
  n.g[0] = a0; n.g[1] = a1; n.g[2] = b0; n.g[3] = b1; n.g[4] = k;
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_box(rt_nw_scene *s, const double p0[3], const double p1[3], int32_t mat) {
  if (!s || !p0 || !p1 || !valid_mat(s, mat)) return set_error(RT_EINVAL, "rt_nw_box: bad argument");
  SNode n;
  n.kind = kBox;
  n.mat = mat;
  for (int a = 0; a < 3; ++a) {
    n.g[a] = p0[a];
    n.g[4 + a] = p1[a];
  }
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_constant_medium(rt_nw_scene *s, int32_t boundary, double density, int32_t tex) {
  if (!s || !valid_node(s, boundary) || !valid_tex(s, tex) || !(density > 0))
    return set_error(RT_EINVAL, "rt_nw_constant_medium: bad argument");
  const int m = rt_nw_mat_isotropic(s, tex);  // phase_function = new isotropic(a) constant_medium.h:12-17
  if (m < 0) return m;
  SNode n;
  n.type = kMediumNode;
  n.child = boundary;
  n.density = density;
  n.phase_mat = m;
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_medium_samples(rt_nw_scene *s, int32_t medium, int32_t samples) {
  if (!s || !valid_node(s, medium) || s->nodes[medium].type != kMediumNode || samples < 1 || samples > 8)
    return set_error(RT_EINVAL, "rt_nw_medium_samples: bad medium or samples not in 1..8");
  s->nodes[medium].samples = samples;
  s->flat_valid = false;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_group(rt_nw_scene *s, const int32_t *objects, int32_t count) {
  if (!s || (count > 0 && !objects) || count < 0) return set_error(RT_EINVAL, "rt_nw_group: bad argument");
  SNode n;
  n.type = kGroup;
  for (int i = 0; i < count; ++i) {
    if (!valid_node(s, objects[i])) return set_error(RT_EINVAL, "rt_nw_group: bad object %d", objects[i]);
    n.kids.push_back(objects[i]);
  }
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_translate(rt_nw_scene *s, int32_t object, const double offset[3]) {
  if (!s || !offset || !valid_node(s, object)) return set_error(RT_EINVAL, "rt_nw_translate: bad argument");
  SNode n;
  n.type = kTranslate;
  n.child = object;
  for (int a = 0; a < 3; ++a) n.off[a] = offset[a];
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_rotate_y(rt_nw_scene *s, int32_t object, double angle_deg) {
  if (!s || !valid_node(s, object) || !std::isfinite(angle_deg)) return set_error(RT_EINVAL, "rt_nw_rotate_y: bad argument");
  SNode n;
  n.type = kRotate;
  n.child = object;
  n.angle = angle_deg;
  return add_node(s, n);
}

RTMI_EXPORT int rt_nw_world_add(rt_nw_scene *s, int32_t object) {
  if (!s || !valid_node(s, object)) return set_error(RT_EINVAL, "rt_nw_world_add: bad object");
  s->world.push_back(object);
  s->flat_valid = false;
  return RT_OK;
}

RTMI_EXPORT int rt_nw_set_background(rt_nw_scene *s, double r, double g, double b) {
  if (!s) return set_error(RT_EINVAL, "null scene");
  s->background[0] = float(r);
  s->background[1] = float(g);
  s->background[2] = float(b);
  return RT_OK;
}

RTMI_EXPORT int rt_nw_scene_grid_stats(rt_nw_scene *s, int32_t *dims3, int32_t *max_cell, int32_t *n_big,
                                       int32_t *n_refs) {
  return rtmi::nw::scene_grid_stats(s, dims3, max_cell, n_big, n_refs);
}

RTMI_EXPORT int rt_nw_scene_flat(rt_nw_scene *s, rt_nw_flat *out) {
  if (!s || !out) return set_error(RT_EINVAL, "null");
  if (int rc = flatten(s)) return rc;
  out->n_obj = int32_t(s->flat_obj.size());
  out->n_inst = int32_t(s->flat_inst.size());
  out->n_mat = int32_t(s->mat.size());
  out->n_tex = int32_t(s->tex.size());
  out->n_perlin = int32_t(s->perlin_perm.size() / (3 * kPerlinN));
  out->n_image = int32_t(s->image.size());
  out->obj = reinterpret_cast<const float *>(s->flat_obj.data());
  out->inst = reinterpret_cast<const float *>(s->flat_inst.data());
  out->mat = reinterpret_cast<const float *>(s->mat.data());
  out->tex = reinterpret_cast<const float *>(s->tex.data());
  out->perlin_vec = s->perlin_vec.data();
  out->perlin_perm = s->perlin_perm.data();
  out->image_desc = reinterpret_cast<const int32_t *>(s->image.data());
  out->image_px = s->image_px.data();
  out->image_bytes = int64_t(s->image_px.size());
  for (int c = 0; c < 3; ++c) out->background[c] = s->background[c];
  return RT_OK;
}

RTMI_EXPORT int rt_nw_xorwow_uniforms(uint64_t seed, int32_t n, float *out) {
  if (n < 0 || (n > 0 && !out)) return set_error(RT_EINVAL, "rt_nw_xorwow_uniforms: bad argument");
  Xorwow g(seed);
  for (int i = 0; i < n; ++i) out[i] = g.uniform();
  return RT_OK;
}

// ---------------------------------------------------------------------------
// The reference's scenes (rt_next_week/cuda/main.cu:163-413, create_world
// main.cu:415-490), drawing from curand_init(1984, 0, 0) (main.cu:103-107).
// ---------------------------------------------------------------------------
namespace {

struct Preset {
  rt_nw_scene *s;
  Xorwow g;
  bool rtl;
  int rc = RT_OK;

  int chk(int v) {
    if (v < 0 && rc == RT_OK) rc = v;
    return v;
  }
  // vec3(f(), f(), f()) with the configured argument evaluation order
  template <class F> void vec3_draw(F f, float out[3]) {
    if (rtl) { out[2] = f(); out[1] = f(); out[0] = f(); }
    else { out[0] = f(); out[1] = f(); out[2] = f(); }
  }
  int solid(double r, double g_, double b) { return chk(rt_nw_tex_solid(s, r, g_, b)); }
  int lam(double r, double g_, double b) { return chk(rt_nw_mat_lambertian(s, solid(r, g_, b))); }
  int lam_t(int tex) { return chk(rt_nw_mat_lambertian(s, tex)); }
  int sphere(double x, double y, double z, double r, int m) {
    const double c[3] = {x, y, z};
    return chk(rt_nw_sphere(s, c, r, m));
  }
  void add(int obj) { chk(rt_nw_world_add(s, obj)); }
  int checker() { return chk(rt_nw_tex_checker(s, solid(0.2, 0.3, 0.1), solid(0.9, 0.9, 0.9))); }
  // perlin::perlin perlin.h:8-21: ranvec = random_vec3(-1, 1), then
  // perm_x, perm_y, perm_z by perlin_generate_perm / permute (perlin.h:92-112)
  int noise(double scale) {
    float ranvec[3 * kPerlinN];
    int32_t perm[3 * kPerlinN];
    for (int i = 0; i < kPerlinN; ++i) vec3_draw([&] { return g.range(-1.f, 1.f); }, ranvec + 3 * i);
    for (int a = 0; a < 3; ++a) {
      int32_t *p = perm + a * kPerlinN;
      for (int i = 0; i < kPerlinN; ++i) p[i] = i;
      for (int i = kPerlinN - 1; i > 0; --i) std::swap(p[i], p[g.rint(kPerlinN)]);
    }
    return chk(rt_nw_tex_noise(s, scale, ranvec, perm));
  }
  int box(double x0, double y0, double z0, double x1, double y1, double z1, int m) {
    const double p0[3] = {x0, y0, z0}, p1[3] = {x1, y1, z1};
    return chk(rt_nw_box(s, p0, p1, m));
  }
  int xf(int obj, double angle, double tx, double ty, double tz) {
    const double off[3] = {tx, ty, tz};
    return chk(rt_nw_translate(s, chk(rt_nw_rotate_y(s, obj, angle)), off));
  }

  // random_scene main.cu:163-213
  void random_scene() {
    add(sphere(0, -1000.0, -1, 1000, lam_t(checker())));
    for (int a = -11; a < 11; a++)
      for (int b = -11; b < 11; b++) {
        const float choose_mat = g.uniform();
        float ctr[3];
        if (rtl) { ctr[2] = float(b) + g.uniform(); ctr[0] = float(a) + g.uniform(); }
        else { ctr[0] = float(a) + g.uniform(); ctr[2] = float(b) + g.uniform(); }
        ctr[1] = 0.2f;
        const double c0[3] = {ctr[0], ctr[1], ctr[2]};
        if (choose_mat < 0.8f) {
          const double c1[3] = {ctr[0], ctr[1] + g.uniform() * 0.5f, ctr[2]};
          float alb[3];
          vec3_draw([&] { const float x = g.uniform(); return x * g.uniform(); }, alb);
          add(chk(rt_nw_moving_sphere(s, c0, c1, 0.0, 1.0, 0.2, lam(alb[0], alb[1], alb[2]))));
        } else if (choose_mat < 0.95f) {
          float alb[3], fuzz;
          if (rtl) {
            fuzz = 0.5f * g.uniform();
            vec3_draw([&] { return 0.5f * (1.0f + g.uniform()); }, alb);
          } else {
            vec3_draw([&] { return 0.5f * (1.0f + g.uniform()); }, alb);
            fuzz = 0.5f * g.uniform();
          }
          add(chk(rt_nw_sphere(s, c0, 0.2, chk(rt_nw_mat_metal(s, solid(alb[0], alb[1], alb[2]), fuzz)))));
        } else {
          add(chk(rt_nw_sphere(s, c0, 0.2, chk(rt_nw_mat_dielectric(s, 1.5)))));
        }
      }
    add(sphere(0, 1, 0, 1.0, chk(rt_nw_mat_dielectric(s, 1.5))));
    add(sphere(-4, 1, 0, 1.0, lam(0.4, 0.2, 0.1)));
    add(sphere(4, 1, 0, 1.0, chk(rt_nw_mat_metal(s, solid(0.7, 0.6, 0.5), 0.0))));
  }
  // two_spheres main.cu:215-226
  void two_spheres() {
    const int m = lam_t(checker());
    add(sphere(0, -10, 0, 10, m));
    add(sphere(0, 10, 0, 10, m));
  }
  // two_perlin_spheres main.cu:228-238
  void two_perlin_spheres() {
    const int m = lam_t(noise(4));
    add(sphere(0, -1000, 0, 1000, m));
    add(sphere(0, 2, 0, 2, m));
  }
  // earth main.cu:240-248
  void earth(const uint8_t *img, int w, int h) {
    add(sphere(0, 0, 0, 2, lam_t(chk(rt_nw_tex_image(s, img, w, h)))));
  }
  // simple_light main.cu:250-266
  void simple_light() {
    const int m = lam_t(noise(4));
    add(sphere(0, -1000, 0, 1000, m));
    add(sphere(0, 2, 0, 2, m));
    add(chk(rt_nw_rect(s, RT_NW_XY, 3, 5, 1, 2, -2, chk(rt_nw_mat_diffuse_light(s, solid(4, 4, 4))))));
    add(sphere(0, 6, 0, 1.5, chk(rt_nw_mat_diffuse_light(s, solid(6, 4, 4)))));
  }
  // cornell_box main.cu:268-299, cornell_smoke main.cu:301-329
  void cornell(bool smoke) {
    const int red = lam(.65, .05, .05), white = lam(.73, .73, .73), green = lam(.12, .45, .15);
    const int light = chk(rt_nw_mat_diffuse_light(s, solid(15, 15, 15)));
    add(chk(rt_nw_rect(s, RT_NW_YZ, 0, 555, 0, 555, 555, green)));
    add(chk(rt_nw_rect(s, RT_NW_YZ, 0, 555, 0, 555, 0, red)));
    add(chk(rt_nw_rect(s, RT_NW_XZ, 213, 343, 227, 332, 554, light)));
    add(chk(rt_nw_rect(s, RT_NW_XZ, 0, 555, 0, 555, 0, white)));
    add(chk(rt_nw_rect(s, RT_NW_XZ, 0, 555, 0, 555, 555, white)));
    add(chk(rt_nw_rect(s, RT_NW_XY, 0, 555, 0, 555, 555, white)));
    int box1 = xf(box(0, 0, 0, 165, 330, 165, white), 15, 265, 0, 295);
    int box2 = xf(box(0, 0, 0, 165, 165, 165, white), -18, 130, 0, 65);
    if (smoke) {
      box1 = chk(rt_nw_constant_medium(s, box1, 0.01, solid(0, 0, 0)));
      box2 = chk(rt_nw_constant_medium(s, box2, 0.01, solid(1, 1, 1)));
    }
    add(box1);
    add(box2);
  }
  // rt_next_week_final_scene main.cu:331-413
  void final_scene(const uint8_t *img, int w, int h) {
    const int ground = lam(0.48, 0.83, 0.53);
    for (int i = 0; i < 20; i++)
      for (int j = 0; j < 20; j++) {
        const float wd = 100.0f;
        const float x0 = -1000.0f + float(i) * wd, z0 = -1000.0f + float(j) * wd, y0 = 0.0f;
        const float x1 = x0 + wd, y1 = g.range(1.f, 101.f), z1 = z0 + wd;
        add(box(x0, y0, z0, x1, y1, z1, ground));
      }
    add(chk(rt_nw_rect(s, RT_NW_XZ, 123, 423, 147, 412, 554, chk(rt_nw_mat_diffuse_light(s, solid(7, 7, 7))))));
    {
      const double c1[3] = {400, 400, 200}, c2[3] = {430, 400, 200};
      add(chk(rt_nw_moving_sphere(s, c1, c2, 0, 1, 50, lam(0.7, 0.3, 0.1))));
    }
    add(sphere(260, 150, 45, 50, chk(rt_nw_mat_dielectric(s, 1.5))));
    add(sphere(0, 150, 145, 50, chk(rt_nw_mat_metal(s, solid(0.8, 0.8, 0.9), 1.0))));
    const int sd2 = sphere(360, 150, 145, 70, chk(rt_nw_mat_dielectric(s, 1.5)));
    add(sd2);
    add(chk(rt_nw_constant_medium(s, sd2, 0.2, solid(0.2, 0.4, 0.9))));
    const int fog = sphere(0, 0, 0, 5000, chk(rt_nw_mat_dielectric(s, 1.5)));
    const int fog_medium = chk(rt_nw_constant_medium(s, fog, 0.0001, solid(1, 1, 1)));
    // The fog's box (r = 5000) sorts first on every axis, so the reference's
    // bvh_node puts it alone in a span-1 leaf (left = right, bvh.h:147-151)
    // that its traversal evaluates twice per ray (bvh.h:90-97): two
    // scattering-distance draws, the last hit wins.
    chk(rt_nw_medium_samples(s, fog_medium, 2));
    add(fog_medium);
    add(sphere(400, 200, 400, 100, lam_t(chk(rt_nw_tex_image(s, img, w, h)))));
    add(sphere(220, 280, 300, 80, lam_t(noise(0.1))));
    const int white = lam(.73, .73, .73);
    std::vector<int32_t> cluster(1000);
    for (int j = 0; j < 1000; j++) {
      float c[3];
      vec3_draw([&] { return g.range(0.f, 165.f); }, c);
      cluster[j] = sphere(c[0], c[1], c[2], 10, white);
    }
    add(xf(chk(rt_nw_group(s, cluster.data(), 1000)), 15, -100, 270, 395));
  }
};

}  // namespace

RTMI_EXPORT int rt_nw_scene_preset(rt_nw_scene *s, int32_t which, const uint8_t *image, int32_t w, int32_t h,
                                   double aspect, uint32_t flags, rt_nw_camera *cam) {
  if (!s || !cam || !(aspect > 0)) return set_error(RT_EINVAL, "rt_nw_scene_preset: bad argument");
  if (which < 1 || which > 8) return set_error(RT_EINVAL, "rt_nw_scene_preset: scene %d not in 1..8", which);
  if (image && (w <= 0 || h <= 0)) return set_error(RT_EINVAL, "rt_nw_scene_preset: bad image size");
  Preset p{s, Xorwow(1984), (flags & RT_NW_ARGS_RTL) != 0};
  // create_world defaults main.cu:421-427, then the per-scene switch
  double lookfrom[3] = {13, 2, 3}, lookat[3] = {0, 0, 0};
  double aperture = 0.0, vfov = 40.0;
  const double sky[3] = {0.70, 0.80, 1.00};
  const double *bg = sky;
  const double black[3] = {0, 0, 0};
  switch (which) {
    case 1: p.random_scene(); vfov = 20.0; aperture = 0.05; break;
    case 2: p.two_spheres(); vfov = 20.0; break;
    case 3: p.two_perlin_spheres(); vfov = 20.0; break;
    case 4: p.earth(image, w, h); break;
    case 5:
      bg = black;
      p.simple_light();
      lookfrom[0] = 26; lookfrom[1] = 3; lookfrom[2] = 6;
      lookat[0] = 0; lookat[1] = 2; lookat[2] = 0;
      vfov = 20.0;
      break;
    case 6: case 7:
      bg = black;
      p.cornell(which == 7);
      lookfrom[0] = 278; lookfrom[1] = 278; lookfrom[2] = -800;
      lookat[0] = 278; lookat[1] = 278; lookat[2] = 0;
      break;
    case 8:
      bg = black;
      p.final_scene(image, w, h);
      lookfrom[0] = 478; lookfrom[1] = 278; lookfrom[2] = -600;
      lookat[0] = 278; lookat[1] = 278; lookat[2] = 0;
      break;
  }
  if (p.rc) return p.rc;
  rt_nw_set_background(s, bg[0], bg[1], bg[2]);
  const double vup[3] = {0, 1, 0};
  const double dx = lookfrom[0] - lookat[0], dy = lookfrom[1] - lookat[1], dz = lookfrom[2] - lookat[2];
  const double dist = std::sqrt(dx * dx + dy * dy + dz * dz);  // main.cu:486
  return rt_nw_camera_init(cam, lookfrom, lookat, vup, vfov, aspect, aperture, dist, 0.0, 1.0);
}
