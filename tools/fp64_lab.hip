// fp64 / integer VALU issue costs and the accuracy of v_rcp_f64 on gfx950 -- the numbers the
// warpPerspective coordinate rewrite rests on (DESIGN K3p).  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fp64_lab.hip -o tools/fp64_lab
//   tools/fp64_lab            (on the GPU box)
// Part 1: cycles per wave64 instruction, 16 independent chains per lane, 4 waves per SIMD.
// Part 2: max relative error of v_rcp_f64 alone and after one Newton step over 2^24 random
//         w in [2^-8, 2^8] (both signs), against the correctly rounded 1 / w (IEEE division).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

constexpr int kIters = 1024;

#define OP64(NAME, ASM)                                                                   \
  __global__ __launch_bounds__(256) void NAME(double* out, double seed) {                 \
    double r[16];                                                                         \
    for (int i = 0; i < 16; ++i) r[i] = seed + i * 0.37 + threadIdx.x * 1e-3;             \
    for (int it = 0; it < kIters; ++it) {                                                 \
      _Pragma("unroll") for (int i = 0; i < 16; ++i)                                      \
        asm volatile(ASM : "+v"(r[i]) : "v"(r[(i + 5) & 15]), "v"(r[(i + 9) & 15]));      \
    }                                                                                     \
    double a = 0;                                                                         \
    for (int i = 0; i < 16; ++i) a += r[i];                                               \
    out[blockIdx.x * 256 + threadIdx.x] = a;                                              \
  }
#define OP32(NAME, ASM)                                                                   \
  __global__ __launch_bounds__(256) void NAME(double* out, double seed) {                 \
    uint32_t r[16];                                                                       \
    for (int i = 0; i < 16; ++i) r[i] = (uint32_t)seed * 7919u + i * 104729u + threadIdx.x; \
    for (int it = 0; it < kIters; ++it) {                                                 \
      _Pragma("unroll") for (int i = 0; i < 16; ++i)                                      \
        asm volatile(ASM : "+v"(r[i]) : "v"(r[(i + 5) & 15]), "v"(r[(i + 9) & 15]));      \
    }                                                                                     \
    uint32_t a = 0;                                                                       \
    for (int i = 0; i < 16; ++i) a ^= r[i];                                               \
    out[blockIdx.x * 256 + threadIdx.x] = a;                                              \
  }
OP64(k_fma_f64, "v_fma_f64 %0, %1, %2, %0")
OP64(k_add_f64, "v_add_f64 %0, %1, %0")
OP64(k_mul_f64, "v_mul_f64 %0, %1, %0")
OP64(k_rcp_f64, "v_rcp_f64 %0, %1")
OP32(k_add_u32, "v_add_u32_e32 %0, %1, %0")
OP32(k_alignbit, "v_alignbit_b32 %0, %1, %2, 30")
OP32(k_bfe_i32, "v_bfe_i32 %0, %1, 0, 21")
OP32(k_and_b32, "v_and_b32_e32 %0, %1, %0")
OP32(k_min_u32, "v_min_u32_e32 %0, %1, %0")
OP32(k_fma_f32, "v_fma_f32 %0, %1, %2, %0")

__global__ void rcp_err(const double* w, int n, double* err0, double* err1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = w[i];
  const double exact = 1.0 / x;  // IEEE division (correctly rounded)
  const double y0 = __builtin_amdgcn_rcp(x);
  const double e = __builtin_fma(-x, y0, 1.0);
  const double y1 = __builtin_fma(y0, e, y0);
  err0[i] = fabs(y0 - exact) / fabs(exact);
  err1[i] = fabs(y1 - exact) / fabs(exact);
}

template <class K>
float time_kernel(K k, double* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = 256 * 4;  // 4 workgroups of 4 waves per CU: 4 waves per SIMD
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.5);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.5);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 1024 * sizeof(double) * 4);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double ghz = clk_khz / 1e6;
  struct {
    const char* name;
    void (*k)(double*, double);
  } ks[] = {{"v_fma_f64", k_fma_f64}, {"v_add_f64", k_add_f64}, {"v_mul_f64", k_mul_f64},
            {"v_rcp_f64", k_rcp_f64}, {"v_add_u32", k_add_u32}, {"v_alignbit_b32", k_alignbit},
            {"v_bfe_i32", k_bfe_i32}, {"v_and_b32", k_and_b32}, {"v_min_u32", k_min_u32},
            {"v_fma_f32", k_fma_f32}};
  printf("clock attribute %.3f GHz; 4 waves per SIMD, 16 independent chains\n", ghz);
  for (auto& k : ks) {
    const float ms = time_kernel(k.k, out);
    // instructions per SIMD: 4 waves x kIters x 16; cycles = ms * 1e-3 * clk
    const double instr = 4.0 * kIters * 16;
    printf("%-16s %8.4f ms  %6.2f cycles per wave instruction (at the attribute clock)\n", k.name, ms,
           ms * 1e-3 * ghz * 1e9 / instr);
  }
  const int n = 1 << 24;
  std::vector<double> w(n);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;  // [0, 1)
    w[i] = std::ldexp(1.0 + u, (int)(s % 17) - 8) * ((s >> 5) & 1 ? 1.0 : -1.0);
  }
  double *dw, *e0, *e1;
  hipMalloc(&dw, n * 8);
  hipMalloc(&e0, n * 8);
  hipMalloc(&e1, n * 8);
  hipMemcpy(dw, w.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(rcp_err, dim3((n + 255) / 256), dim3(256), 0, 0, dw, n, e0, e1);
  std::vector<double> h0(n), h1(n);
  hipMemcpy(h0.data(), e0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), e1, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0;
  for (int i = 0; i < n; ++i) {
    m0 = std::fmax(m0, h0[i]);
    m1 = std::fmax(m1, h1[i]);
  }
  printf("v_rcp_f64 max relative error over %d w: %.3e (2^%.2f); after one Newton step: %.3e (2^%.2f)\n", n, m0,
         std::log2(m0 > 0 ? m0 : 1e-300), m1, std::log2(m1 > 0 ? m1 : 1e-300));
  return 0;
}
