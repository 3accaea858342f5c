// tools/nw_order_sim.cpp — host-only model of the Next-Week object BVH walk
// (analysis; not product): node box tests per ray for the kernel's fixed DFS
// order (stackless skip links) against a near-child-first order (stack walk,
// the child whose centre lies first along the ray visited first), over camera
// rays and one bounce of random directions from their hit points.  Object hits:
// exact for plain spheres and boxes; an instanced or moving object counts as
// hit where the ray enters its leaf box (an approximation shared by both orders).
// Build (from a_dive_into_ray_tracing_amd/csrc):
//   g++ -O2 -std=c++17 -w -I. -o /tmp/nw_order_sim ../../tools/nw_order_sim.cpp rtmi_nw_scene.cpp rtmi_host.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../a_dive_into_ray_tracing_amd/csrc/rtmi_nw_internal.h"

using namespace rtmi::nw;

static DeviceScene ds;
static std::vector<int> left_, right_;

static bool slab(const float *lo, const float *hi, const double o[3], const double ix[3], double tmax, double &tn) {
  double t0 = 0, t1 = tmax;
  for (int a = 0; a < 3; ++a) {
    double u = (lo[a] - o[a]) * ix[a], v = (hi[a] - o[a]) * ix[a];
    if (u > v) std::swap(u, v);
    t0 = std::max(t0, u);
    t1 = std::min(t1, v);
  }
  tn = t0;
  return t0 <= t1;
}

static void test_leaf(int n, const double o[3], const double d[3], const double ix[3], double &tmax, long &tests) {
  const Node &nd = ds.nodes[n];
  for (int k = nd.leaf >> 4; k < (nd.leaf >> 4) + (nd.leaf & 15); ++k) {
    ++tests;
    const Obj &ob = ds.obj[k];
    if (ob.kind == kSphere && ob.inst < 0) {
      const double c[3] = {ob.g0[0], ob.g0[1], ob.g0[2]}, r = ob.g0[3];
      const double oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
      const double A = d[0] * d[0] + d[1] * d[1] + d[2] * d[2], B = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
      const double C = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - r * r, disc = B * B - A * C;
      if (disc > 0) {
        double t = (-B - std::sqrt(disc)) / A;
        if (!(t > 0.001)) t = (-B + std::sqrt(disc)) / A;
        if (t > 0.001 && t < tmax) tmax = t;
      }
    } else if (ob.kind == kBox && ob.inst < 0) {
      double tn;
      if (slab(ob.g0, ob.g1, o, ix, tmax, tn) && tn > 0.001) tmax = tn;
    } else {
      double tn;
      if (slab(nd.bmin, nd.bmax, o, ix, tmax, tn) && tn > 0.001) tmax = tn;
    }
  }
}

static void walk_dfs(const double o[3], const double d[3], long &visits, long &tests, double &tmax) {
  double ix[3];
  for (int a = 0; a < 3; ++a) ix[a] = 1.0 / (std::fabs(d[a]) < 1e-20 ? 1e-20 : d[a]);
  int node = 0;
  while (node < int(ds.nodes.size())) {
    const Node &n = ds.nodes[node];
    double tn;
    const bool enter = slab(n.bmin, n.bmax, o, ix, tmax, tn);
    ++visits;
    if (enter && n.leaf >= 0) test_leaf(node, o, d, ix, tmax, tests);
    node = enter ? node + 1 : n.skip;
  }
}

static void walk_ordered(const double o[3], const double d[3], long &visits, long &tests, double &tmax) {
  double ix[3];
  for (int a = 0; a < 3; ++a) ix[a] = 1.0 / (std::fabs(d[a]) < 1e-20 ? 1e-20 : d[a]);
  int stack[128], sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const int node = stack[--sp];
    const Node &n = ds.nodes[node];
    double tn;
    ++visits;
    if (!slab(n.bmin, n.bmax, o, ix, tmax, tn)) continue;
    if (n.leaf >= 0) { test_leaf(node, o, d, ix, tmax, tests); continue; }
    const int a = left_[node], b = right_[node];
    // near first: the child whose box centre projects first on the ray
    double pa = 0, pb = 0;
    for (int k = 0; k < 3; ++k) {
      pa += (ds.nodes[a].bmin[k] + ds.nodes[a].bmax[k]) * d[k];
      pb += (ds.nodes[b].bmin[k] + ds.nodes[b].bmax[k]) * d[k];
    }
    if (pa <= pb) { stack[sp++] = b; stack[sp++] = a; }
    else { stack[sp++] = a; stack[sp++] = b; }
  }
}

int main(int argc, char **argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 8;
  rt_nw_scene *s = nullptr;
  rt_nw_camera cam;
  rt_nw_scene_create(&s);
  if (rt_nw_scene_preset(s, which, nullptr, 0, 0, 1.0, 0, &cam)) return 1;
  if (build_device_scene(s, ds)) return 1;
  const int nn = int(ds.nodes.size());
  left_.assign(nn, -1);
  right_.assign(nn, -1);
  for (int i = 0; i < nn; ++i)
    if (ds.nodes[i].leaf < 0) { left_[i] = i + 1; right_[i] = ds.nodes[i + 1].skip; }
  const auto &c = cam.cam;
  long v[2][2] = {{0, 0}, {0, 0}}, t[2][2] = {{0, 0}, {0, 0}}, rays[2] = {0, 0};
  srand(7);
  for (int j = 0; j < 100; ++j)
    for (int i = 0; i < 100; ++i) {
      const double u = (i + 0.5) / 100, w = (j + 0.5) / 100;
      double o[3], d[3];
      for (int a = 0; a < 3; ++a) {
        o[a] = c.origin[a];
        d[a] = c.lower_left_corner[a] + u * c.horizontal[a] + w * c.vertical[a] - o[a];
      }
      double tm0 = INFINITY, tm1 = INFINITY;
      walk_dfs(o, d, v[0][0], t[0][0], tm0);
      walk_ordered(o, d, v[0][1], t[0][1], tm1);
      ++rays[0];
      if (!std::isfinite(tm0)) continue;
      // one bounce: a random direction from the hit point
      double p[3], nd[3], len = 0;
      for (int a = 0; a < 3; ++a) { p[a] = o[a] + tm0 * d[a] * 0.999; nd[a] = 2.0 * rand() / RAND_MAX - 1.0; len += nd[a] * nd[a]; }
      if (len < 1e-6) continue;
      tm0 = tm1 = INFINITY;
      walk_dfs(p, nd, v[1][0], t[1][0], tm0);
      walk_ordered(p, nd, v[1][1], t[1][1], tm1);
      ++rays[1];
    }
  printf("scene %d: %d nodes, %zu objects\n", which, nn, ds.obj.size());
  const char *nm[2] = {"camera rays", "one bounce"};
  for (int k = 0; k < 2; ++k)
    printf("  %-12s %6ld rays: DFS %.2f node tests %.2f objects | near-first %.2f node tests %.2f objects\n", nm[k],
           rays[k], double(v[k][0]) / rays[k], double(t[k][0]) / rays[k], double(v[k][1]) / rays[k],
           double(t[k][1]) / rays[k]);
  return 0;
}
