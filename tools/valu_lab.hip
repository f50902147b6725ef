// VALU issue-rate lab (gfx950): cycles per wave64 VALU instruction for the top-2
// selection ops of the K1 matcher epilogue, integer vs float forms, at 1..8 waves per
// SIMD.  Each thread runs 8 independent (b1, b2) chains over a stream of keys:
//   int  : key = v_lshl_add_u32(a, 9, q); b2 = v_med3_u32(b1, b2, key); b1 = v_min_u32(b1, key)
//   float: b2 = v_med3_f32(b1, b2, v);     b1 = v_min_f32(b1, v)
// Reports wall-clock ns per instruction per SIMD and the implied cycles at the measured
// in-kernel clock (s_memtime / s_memrealtime).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_lab tools/valu_lab.hip && ./tools/valu_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 4096;

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t minu(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_min_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t lshladd(uint32_t a, uint32_t q) {
  uint32_t r;
  asm volatile("v_lshl_add_u32 %0, %1, 9, %2" : "=v"(r) : "v"(a), "v"(q));
  return r;
}
__device__ __forceinline__ float med3f(float a, float b, float c) {
  float r;
  asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float minf_(float a, float b) {
  float r;
  asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// MODE 0: int triple (3 VALU / key); MODE 1: float pair (2 VALU / key); MODE 2: int pair
// (med3 + min only, 2 VALU / key)
template <int MODE>
__global__ __launch_bounds__(256) void lab(uint32_t* out, unsigned long long* clk) {
  uint32_t b1[8], b2[8], k[8];
  for (int i = 0; i < 8; ++i) {
    b1[i] = 0x7f000000u - threadIdx.x;
    b2[i] = 0x7f000001u;
    k[i] = 0x40000000u + 977u * (threadIdx.x + 13 * i);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (MODE == 0) {
        const uint32_t key = lshladd(k[i], b1[(i + 1) & 7]);
        b2[i] = med3u(b1[i], b2[i], key);
        b1[i] = minu(b1[i], key);
      } else if constexpr (MODE == 1) {
        const float v = __uint_as_float(k[(i + 3) & 7]);
        b2[i] = __float_as_uint(med3f(__uint_as_float(b1[i]), __uint_as_float(b2[i]), v));
        b1[i] = __float_as_uint(minf_(__uint_as_float(b1[i]), v));
      } else {
        b2[i] = med3u(b1[i], b2[i], k[(i + 3) & 7]);
        b1[i] = minu(b1[i], k[(i + 3) & 7]);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc ^= b1[i] ^ b2[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int MODE>
void run(const char* name, int waves_per_simd, int ninst_per_key) {
  const int blocks = 256 * waves_per_simd;  // 256-thread blocks: one wave per SIMD each
  uint32_t* out;
  unsigned long long* clk;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&clk, (size_t)blocks * 16);
  hipLaunchKernelGGL(lab<MODE>, dim3(blocks), dim3(256), 0, 0, out, clk);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(lab<MODE>, dim3(blocks), dim3(256), 0, 0, out, clk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> c((size_t)2 * blocks);
  hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks; ++i) {
    cyc += (double)c[2 * i];
    rt += (double)c[2 * i + 1];
  }
  const double ghz = cyc / rt * 0.1;  // s_memrealtime ticks at 100 MHz
  const double insts_per_simd = (double)waves_per_simd * kIters * 8 * ninst_per_key;
  const double ns = ms * 1e6;
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
         "\"cycles_per_inst_per_simd\": %.3f}\n",
         name, waves_per_simd, ms, ghz, ns * ghz / insts_per_simd);
  hipFree(out);
  hipFree(clk);
}

int main() {
  for (int w : {1, 2, 3, 4, 8}) {
    run<0>("int lshl_add+med3+min", w, 3);
    run<2>("int med3+min", w, 2);
    run<1>("f32 med3+min", w, 2);
  }
  return 0;
}
