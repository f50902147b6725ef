// Ablation lab for the warp kernel (not part of the library).  Build on this host:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude tools/warp_lab.hip -o tools/warp_lab
// Run on the GPU box: tools/warp_lab [frames]
#include <cmath>
#include <cstdio>
#include <vector>

#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"
namespace kcmc {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
int fail(int c, const std::string& m) { set_error(m); return c; }
int hip_check(hipError_t e, const char* w) { if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e)); return KCMC_EHIP; } return 0; }
int launch_check(const char* w) { return hip_check(hipGetLastError(), w); }
}  // namespace kcmc
#include "../keypoint-consensus-motion-correction_amd/csrc/warp.hip"

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int V>
float run(const uint16_t* src, uint16_t* dst, const double* M, int F, int H, int W, int reps) {
  dim3 grid(kcmc::ceil_div(W, kTileW), kcmc::ceil_div(H, kTileH), F);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((warp_affine_u16_kernel<1, V>), grid, dim3(kThreads), 0, 0, src, dst, M, H, W, 0);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((warp_affine_u16_kernel<1, V>), grid, dim3(kThreads), 0, 0, src, dst, M, H, W, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 2000, H = 1080, W = 1920, reps = 5;
  const size_t n = (size_t)F * H * W;
  uint16_t *src, *dst;
  double* M;
  CK(hipMalloc(&src, n * 2));
  CK(hipMalloc(&dst, n * 2));
  CK(hipMemset(src, 0x5a, n * 2));
  std::vector<double> hm((size_t)F * 6);
  for (int f = 0; f < F; ++f) {
    double th = 0.008 * std::sin(f * 0.7), c = std::cos(th), s = std::sin(th);
    double* m = &hm[(size_t)f * 6];
    m[0] = c; m[1] = -s; m[2] = 4 * std::sin(f * 1.3); m[3] = s; m[4] = c; m[5] = 4 * std::cos(f * 0.9);
  }
  CK(hipMalloc(&M, hm.size() * 8));
  CK(hipMemcpy(M, hm.data(), hm.size() * 8, hipMemcpyHostToDevice));
  const double gb = 2.0 * n * 2 / 1e9;
  const char* names[] = {"full", "no-compute(zeros after staging)", "no-staging-loads", "stores-only",
                         "aligned-u16-taps"};
  float t[5] = {run<0>(src, dst, M, F, H, W, reps), run<1>(src, dst, M, F, H, W, reps),
                run<2>(src, dst, M, F, H, W, reps), run<3>(src, dst, M, F, H, W, reps),
                run<4>(src, dst, M, F, H, W, reps)};
  for (int v = 0; v < 5; ++v) printf("%-34s %8.3f ms  %7.1f GB/s (algorithmic r+w)\n", names[v], t[v], gb / (t[v] * 1e-3));
  // plain copy of the same bytes: the HBM reference point on this box
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n / 8);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n / 8);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-34s %8.3f ms  %7.1f GB/s\n", "uint4 copy", ms / reps, gb / (ms / reps * 1e-3));
  return 0;
}
