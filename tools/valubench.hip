// tools/valubench.hip — measured FP32 VALU ceiling on this MI355X (the
// roofline's denominator check): independent v_fma_f32 chains with VGPR-only
// operands, with one SGPR operand (the form of the sphere loop), packed
// v_pk_fma_f32, and the in-kernel shader clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kChains = 8;

template <int MODE>
__global__ __launch_bounds__(256) void fma_kernel(float *out, int iters, float s0, float s1,
                                                  unsigned long long *clk) {
  float x[kChains];
  for (int c = 0; c < kChains; c++) x[c] = threadIdx.x * 1e-3f + c;
  const float a = 1.0000001f, b = 1e-7f;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  float y = s0;  // uniform (SGPR) operand
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int c = 0; c < kChains; c++) {
        if constexpr (MODE == 0) x[c] = __builtin_fmaf(x[c], a, b);       // VGPR + inline constants
        else if constexpr (MODE == 1) x[c] = __builtin_fmaf(x[c], y, b);  // one SGPR operand
        else x[c] = __builtin_fmaf(x[c], y, s1);                          // two SGPR operands (illegal -> moves)
      }
    }
    y += 1e-9f;
  }
  if (threadIdx.x == 0) {
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
  }
  float s = 0;
  for (int c = 0; c < kChains; c++) s += x[c];
  if (s == 12345.f) out[0] = s;
}

typedef float float2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void pk_kernel(float *out, int iters) {
  float2v x[kChains / 2];
  for (int c = 0; c < kChains / 2; c++) x[c] = float2v{threadIdx.x * 1e-3f + c, c * 0.5f};
  const float2v a = {1.0000001f, 1.0000002f}, b = {1e-7f, 2e-7f};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int c = 0; c < kChains / 2; c++) x[c] = __builtin_elementwise_fma(x[c], a, b);
    }
  }
  float s = 0;
  for (int c = 0; c < kChains / 2; c++) s += x[c].x + x[c].y;
  if (s == 12345.f) out[0] = s;
}

int main() {
  float *out;
  unsigned long long *clk;
  (void)hipMalloc(&out, 4);
  (void)hipMalloc(&clk, 16);
  const int blocks = 256 * 8 * 4, threads = 256, iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto report = [&](const char *name, float ms, double fma_per_thread) {
    const double flops = double(blocks) * threads * fma_per_thread * 2;
    unsigned long long c[2] = {0, 0};
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"TFLOPs\": %.1f, \"clock_GHz\": %.3f}\n", name, ms, flops / ms / 1e9,
           c[1] ? double(c[0]) / double(c[1]) * 0.1 : 0.0);
  };
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(fma_kernel<0>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001f, 1e-7f, clk);
      if (mode == 1) hipLaunchKernelGGL(fma_kernel<1>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001f, 1e-7f, clk);
      if (mode == 2) hipLaunchKernelGGL(fma_kernel<2>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001f, 1e-7f, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) report(mode == 0 ? "fma vgpr" : mode == 1 ? "fma 1 sgpr" : "fma 2 sgpr", ms, double(iters) * 8 * kChains);
    }
  }
  for (int rep = 0; rep < 2; rep++) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(pk_kernel, dim3(blocks), dim3(threads), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep == 1) report("pk_fma", ms, double(iters) * 8 * kChains);
  }
  return 0;
}
