// tools/loopbench.hip — microbenchmark of the brute-force sphere loop alone
// (hit_world_grouped from rtmi_path.h) on the final scene with random rays.
// Measures ray-sphere tests per second for loop variants, to separate the
// loop's ceiling from the shading/regeneration overhead of render_kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
//         -I a_dive_into_ray_tracing_amd/csrc tools/loopbench.hip \
//         -L a_dive_into_ray_tracing_amd/lib -lrtmi -o tools/loopbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "rtmi_path.h"

using namespace rtmi;

__device__ inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ inline float u01(uint32_t &s) { s = hash32(s + 0x9e3779b9U); return float(s >> 8) * 0x1p-24f; }

template <int GP>
__global__ __launch_bounds__(256) void packed_kernel(const SpherePair *__restrict__ pairs, int npairs, int reps,
                                                     unsigned long long *__restrict__ sink) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  V3<float> o = mk(-11.f + 24.f * u01(s), 0.05f + 2.f * u01(s), -11.f + 24.f * u01(s));
  V3<float> d = mk(2.f * u01(s) - 1.f, 2.f * u01(s) - 1.f, 2.f * u01(s) - 1.f);
  unsigned acc = 0;
  for (int r = 0; r < reps; r++) {
    float t;
    int k = hit_world_packed<GP>(pairs, npairs, o, d, t
#if RTMI_STATS
                                 , nullptr
#endif
    );
    acc += unsigned(k);
    o.x += 1e-3f;
    d.y = -d.y;
  }
  if (acc == 0xffffffffu) sink[0] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 7) {
    sink[1] = __builtin_amdgcn_s_memtime() - t0;
    sink[2] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int G, bool PIPE>
__global__ __launch_bounds__(256) void loop_kernel(const float4 *__restrict__ geom, int n, int reps,
                                                   unsigned long long *__restrict__ sink) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  // origins around the camera and in the sphere field; directions random
  V3<float> o = mk(-11.f + 24.f * u01(s), 0.05f + 2.f * u01(s), -11.f + 24.f * u01(s));
  V3<float> d = mk(2.f * u01(s) - 1.f, 2.f * u01(s) - 1.f, 2.f * u01(s) - 1.f);
  unsigned acc = 0;
  for (int r = 0; r < reps; r++) {
    float t;
    int k;
    if constexpr (PIPE) k = hit_world_pipelined<G>(geom, n, o, d, t);
    else k = hit_world_grouped<G>(geom, n, o, d, t
#if RTMI_STATS
                                  , nullptr
#endif
      );
    acc += unsigned(k);
    o.x += 1e-3f;  // a different ray each repetition
    d.y = -d.y;
  }
  if (acc == 0xffffffffu) sink[0] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 32;
  std::vector<double> g(4 * 600), m(4 * 600);
  std::vector<int32_t> kd(600);
  int32_t n = 0;
  rt_scene_random(1, g.data(), kd.data(), m.data(), 600, &n);
  std::vector<float4> geom(n + kGeomPad, make_float4(0, 0, 0, 0));
  for (int k = 0; k < n; k++) {
    float cx = float(g[4 * k]), cy = float(g[4 * k + 1]), cz = float(g[4 * k + 2]), r = float(g[4 * k + 3]);
    geom[k] = make_float4(cx, cy, cz, float(double(cx) * cx + double(cy) * cy + double(cz) * cz - double(r) * r));
  }
  const int n_pad = (n + 15) / 16 * 16;  // multiple of 2*GP for GP <= 8
  std::vector<SpherePair> pairs(n_pad / 2 + 8);  // + prefetch padding
  for (auto &p : pairs) { p.cx = f2v{0, 0}; p.cy = f2v{0, 0}; p.cz = f2v{0, 0}; p.S = f2v{kDummyS, kDummyS}; }
  for (int k = 0; k < n_pad; k++) {
    float4 v = k < n ? geom[k] : make_float4(0, 0, 0, kDummyS);
    SpherePair &p = pairs[k / 2];
    if (k % 2 == 0) { p.cx.x = v.x; p.cy.x = v.y; p.cz.x = v.z; p.S.x = v.w; }
    else { p.cx.y = v.x; p.cy.y = v.y; p.cz.y = v.z; p.S.y = v.w; }
  }
  SpherePair *dp;
  (void)hipMalloc(&dp, pairs.size() * sizeof(SpherePair));
  (void)hipMemcpy(dp, pairs.data(), pairs.size() * sizeof(SpherePair), hipMemcpyHostToDevice);
  float4 *dg;
  unsigned long long *sink;
  hipMalloc(&dg, geom.size() * sizeof(float4));
  hipMalloc(&sink, 32);
  hipMemcpy(dg, geom.data(), geom.size() * sizeof(float4), hipMemcpyHostToDevice);
  const int threads = 256, blocks = 256 * 24;  // ~6 blocks per CU resident, several waves of blocks
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char *name, bool packed = false) {
    if (packed) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, (const float4 *)dp, n_pad / 2, 2, sink);
    else hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dg, n, 2, sink);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int it = 0; it < 3; it++) {
      hipEventRecord(e0);
      if (packed) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, (const float4 *)dp, n_pad / 2, reps, sink);
      else hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, dg, n, reps, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double tests = double(blocks) * threads * reps * n;
    unsigned long long c[3] = {0, 0, 0};
    (void)hipMemcpy(c, sink, 24, hipMemcpyDeviceToHost);
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"Gtests_per_s\": %.1f, \"fp32_TFLOPs_alg18\": %.2f, \"clock_GHz\": %.3f}\n", name, best,
           tests / best / 1e6, tests * 18 / best / 1e9, c[2] ? double(c[1]) / double(c[2]) * 0.1 : 0.0);
  };
  run(loop_kernel<4, false>, "G4");
  run(loop_kernel<8, false>, "G8");
  run(loop_kernel<4, true>, "pipe G4");
  run(loop_kernel<8, true>, "pipe G8");
  run(loop_kernel<2, true>, "pipe G2");
  run(reinterpret_cast<void (*)(const float4 *, int, int, unsigned long long *)>(packed_kernel<2>), "packed GP2", true);
  run(reinterpret_cast<void (*)(const float4 *, int, int, unsigned long long *)>(packed_kernel<4>), "packed GP4", true);
  run(reinterpret_cast<void (*)(const float4 *, int, int, unsigned long long *)>(packed_kernel<8>), "packed GP8", true);
  return 0;
}
