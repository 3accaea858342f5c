// tools/valubench2.hip — issue rate of the exact VALU forms the sphere loop
// can use (inline asm, 8 independent chains, 8 waves/SIMD):
//   A  v_fma_f32    v, s, v, v      (SGPR operand: today's loop)
//   B  v_fma_f32    v, v, v, v      (all VGPR)
//   C  v_pk_fma_f32 v[2], s[2], v[2] with op_sel_hi broadcast of a VGPR
//   D  v_pk_fma_f32 all VGPR pairs
//   E  v_fmac_f32   v, s, v         (VOP2, SGPR src0)
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, int iters, float sa, float sb) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  float va = 1.0000001f + threadIdx.x * 1e-12f, vb = 1e-7f;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {x0, x1}, p1 = {x2, x3}, p2 = {x4, x5}, p3 = {x6, x7};
  f2 pa = {va, va};
  f2 ps = {sa, sb};  // uniform -> SGPR pair
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      if constexpr (MODE == 0) {
#define A(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "s"(sa), "v"(va));
        A(x0) A(x1) A(x2) A(x3) A(x4) A(x5) A(x6) A(x7)
      } else if constexpr (MODE == 1) {
#define B(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(vb), "v"(va));
        B(x0) B(x1) B(x2) B(x3) B(x4) B(x5) B(x6) B(x7)
      } else if constexpr (MODE == 2) {
#define Cc(p) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p) : "v"(pa), "s"(ps));
        Cc(p0) Cc(p1) Cc(p2) Cc(p3) Cc(p0) Cc(p1) Cc(p2) Cc(p3)
      } else if constexpr (MODE == 3) {
#define D(p) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p) : "v"(pa), "v"(pa));
        D(p0) D(p1) D(p2) D(p3) D(p0) D(p1) D(p2) D(p3)
      } else {
#define E(x) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x) : "s"(sa), "v"(va));
        E(x0) E(x1) E(x2) E(x3) E(x4) E(x5) E(x6) E(x7)
      }
    }
  }
  float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + p0.x + p1.x + p2.x + p3.x + p0.y + p1.y + p2.y + p3.y;
  if (s == 12345.f) out[0] = s;
}

int main() {
  float *out;
  (void)hipMalloc(&out, 4);
  const int blocks = 256 * 8 * 4, threads = 256, iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char *names[5] = {"A fma v,s,v,v", "B fma v,v,v,v", "C pk_fma s-pair", "D pk_fma vgpr", "E fmac v,s,v"};
  void (*kern[5])(float *, int, float, float) = {k<0>, k<1>, k<2>, k<3>, k<4>};
  for (int m = 0; m < 5; m++) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(kern[m], dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001f, 1e-7f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    const double instr = double(blocks) * threads / 64 * iters * 64;  // wave-instructions
    const double fmas = instr * 64 * ((m == 2 || m == 3) ? 2 : 1);
    printf("{\"form\": \"%s\", \"ms\": %.3f, \"wave_instr_per_ns\": %.1f, \"TFLOPs\": %.1f, \"cycles_per_instr_per_simd_at_2.4GHz\": %.2f}\n",
           names[m], best, instr / best / 1e6, fmas * 2 / best / 1e9, 1024 * 2.4e9 / (instr / (best * 1e-3)));
  }
  return 0;
}
