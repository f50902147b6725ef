#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int kIters = 2048;
#define OP(NAME, ASM)                                                          \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, int seed) {      \
    uint32_t r[16];                                                            \
    for (int i = 0; i < 16; ++i) r[i] = seed * 7919u + i * 104729u + threadIdx.x; \
    for (int it = 0; it < kIters; ++it) {                                      \
      _Pragma("unroll") for (int i = 0; i < 16; ++i)                           \
        asm volatile(ASM : "+v"(r[i]) : "v"(r[(i + 5) & 15]), "v"(r[(i + 9) & 15])); \
    }                                                                          \
    uint32_t a = 0;                                                            \
    for (int i = 0; i < 16; ++i) a ^= r[i];                                    \
    out[blockIdx.x * 256 + threadIdx.x] = a;                                   \
  }
OP(k_min_u32_e32, "v_min_u32_e32 %0, %1, %0")
OP(k_add_u32_e32, "v_add_u32_e32 %0, %1, %0")
OP(k_sub_u32_e32, "v_sub_u32_e32 %0, %1, %0")
OP(k_med3_u32, "v_med3_u32 %0, %1, %2, %0")
OP(k_lshl_add_u32, "v_lshl_add_u32 %0, %1, 9, %2")
OP(k_min3_u32, "v_min3_u32 %0, %1, %2, %0")
OP(k_add_f32_e32, "v_add_f32_e32 %0, %1, %0")
OP(k_mul_f32_e32, "v_mul_f32_e32 %0, %1, %0")
OP(k_fma_f32, "v_fma_f32 %0, %1, %2, %0")
OP(k_min_f32_e32, "v_min_f32_e32 %0, %1, %0")
OP(k_med3_f32, "v_med3_f32 %0, %1, %2, %0")
OP(k_max_i32_e32, "v_max_i32_e32 %0, %1, %0")
OP(k_pk_min_u16, "v_pk_min_u16 %0, %1, %0")
OP(k_pk_add_u16, "v_pk_add_u16 %0, %1, %0")
OP(k_pk_max_i16, "v_pk_max_i16 %0, %1, %0")
OP(k_and_b32_e32, "v_and_b32_e32 %0, %1, %0")
OP(k_xor_b32_e32, "v_xor_b32_e32 %0, %1, %0")
OP(k_lshlrev_b32_e32, "v_lshlrev_b32_e32 %0, 9, %0")
OP(k_and_or_b32, "v_and_or_b32 %0, %1, %2, %0")
OP(k_lshl_or_b32, "v_lshl_or_b32 %0, %1, 9, %2")
OP(k_add3_u32, "v_add3_u32 %0, %1, %2, %0")
OP(k_perm_b32, "v_perm_b32 %0, %1, %2, %0")
OP(k_alignbit_b32, "v_alignbit_b32 %0, %1, %2, 16")
OP(k_bfe_u32, "v_bfe_u32 %0, %1, 5, 5")
OP(k_cndmask_b32_e32, "v_cndmask_b32_e32 %0, %1, %0, vcc")
OP(k_mul_u32_u24, "v_mul_u32_u24_e32 %0, %1, %0")
OP(k_mad_u32_u24, "v_mad_u32_u24 %0, %1, %2, %0")
OP(k_cvt_f32_u32, "v_cvt_f32_u32_e32 %0, %1")
OP(k_dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %2, %0")
OP(k_mov_b32_e32, "v_mov_b32_e32 %0, %1")
OP(k_cvt_pk_u16_u32, "v_cvt_pk_u16_u32 %0, %1, %2")
OP(k_max_u16, "v_max_u16_e32 %0, %1, %0")
typedef void (*KF)(uint32_t*, int);
void run(const char* name, KF k, int w, int pk) {
  const int blocks = 256 * w;
  uint32_t* out; hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 2);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double inst = (double)w * kIters * 16;  // per SIMD
  printf("%-16s w=%d  ns/inst/SIMD=%.3f  cycles@2.1GHz=%.2f\n", name, w, ms * 1e6 / inst, ms * 1e6 / inst * 2.1);
  hipFree(out);
}
int main() {
  struct { const char* n; KF k; } ks[] = {{"min_u32_e32", k_min_u32_e32}, {"add_u32_e32", k_add_u32_e32}, {"sub_u32_e32", k_sub_u32_e32}, {"med3_u32", k_med3_u32}, {"lshl_add_u32", k_lshl_add_u32}, {"min3_u32", k_min3_u32}, {"add_f32_e32", k_add_f32_e32}, {"mul_f32_e32", k_mul_f32_e32}, {"fma_f32", k_fma_f32}, {"min_f32_e32", k_min_f32_e32}, {"med3_f32", k_med3_f32}, {"max_i32_e32", k_max_i32_e32}, {"pk_min_u16", k_pk_min_u16}, {"pk_add_u16", k_pk_add_u16}, {"pk_max_i16", k_pk_max_i16}, {"and_b32_e32", k_and_b32_e32}, {"xor_b32_e32", k_xor_b32_e32}, {"lshlrev_b32_e32", k_lshlrev_b32_e32}, {"and_or_b32", k_and_or_b32}, {"lshl_or_b32", k_lshl_or_b32}, {"add3_u32", k_add3_u32}, {"perm_b32", k_perm_b32}, {"alignbit_b32", k_alignbit_b32}, {"bfe_u32", k_bfe_u32}, {"cndmask_b32_e32", k_cndmask_b32_e32}, {"mul_u32_u24", k_mul_u32_u24}, {"mad_u32_u24", k_mad_u32_u24}, {"cvt_f32_u32", k_cvt_f32_u32}, {"dot2_u32_u16", k_dot2_u32_u16}, {"mov_b32_e32", k_mov_b32_e32}, {"cvt_pk_u16_u32", k_cvt_pk_u16_u32}, {"max_u16", k_max_u16}};
  for (auto& e : ks) run(e.n, e.k, 8, 0);
}
