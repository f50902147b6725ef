// Ablation lab for the warp kernel (not part of the library).  Build on this host:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude tools/warp_lab.hip -o tools/warp_lab
// Run on the GPU box: tools/warp_lab [frames] [texture.u16]
// (texture.u16: one raw 1080 x 1920 uint16 frame, e.g. the bench texture written by
//  tools/write_texture.py; adds a fifth source-value set, every frame = that texture)
#include <cmath>
#include <cstdio>
#include <vector>

#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"
namespace kcmc {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
int fail(int c, const std::string& m) { set_error(m); return c; }
int hip_check(hipError_t e, const char* w) { if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e)); return KCMC_EHIP; } return 0; }
int launch_check(const char* w) { return hip_check(hipGetLastError(), w); }
int workspace_alloc(kcmc_ctx*, void**, size_t, hipStream_t) { return KCMC_EUNSUPPORTED; }
int workspace_free(kcmc_ctx*, void*, hipStream_t, size_t) { return KCMC_EUNSUPPORTED; }
}  // namespace kcmc
// -DWARP_SRC='"path"' builds the lab against another version of warp.hip (A/B on one box)
#ifndef WARP_SRC
#define WARP_SRC "../keypoint-consensus-motion-correction_amd/csrc/warp.hip"
#endif
#include WARP_SRC

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__global__ void fill_kernel(uint16_t* a, size_t n, uint32_t dist) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    uint32_t v = h >> 16;
    if (dist == 0) v &= 0x3fff;
    if (dist == 1) v = (h & 1023) == 0 ? 60000 : (v & 0x1fff);
    if (dist == 3) {  // bright blobs: 1 in 8 of the 32 x 32 blocks of a 1920-wide frame near 40k
      const size_t px = i % (1080 * 1920), bx = (px % 1920) >> 5, by = (px / 1920) >> 5;
      uint32_t hb = (uint32_t)(bx * 73856093u ^ by * 19349663u ^ (i / (1080 * 1920)) * 83492791u);
      hb ^= hb >> 13;
      hb *= 0x5bd1e995u;
      v = ((hb >> 24) & 7) == 0 ? 36000 + (v & 0x1fff) : (v & 0x1fff);
    }
    a[i] = (uint16_t)v;
  }
}

__global__ void tiny_kernel(unsigned* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[1] = p[0] + 1;
}

__global__ void diff_kernel(const uint16_t* a, const uint16_t* b, size_t n, unsigned long long* cnt) {
  unsigned long long c = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

// order-sensitive checksum of an output stack (compares the outputs of two lab builds)
__global__ void hash_kernel(const uint16_t* a, size_t n, unsigned long long* h) {
  unsigned long long c = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += (unsigned long long)a[i] * (2654435761ull * (i + 1) | 1ull);
  atomicAdd(h, c);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <class L>
float timeit(L launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 2000, H = 1080, W = 1920, reps = 5;
  const size_t n = (size_t)F * H * W;
  uint16_t *src, *dst, *dst2;
  double* M;
  unsigned long long* cnt;
  CK(hipMalloc(&src, n * 2));
  CK(hipMalloc(&dst, n * 2));
  CK(hipMalloc(&dst2, n * 2));
  CK(hipMalloc(&cnt, 8));
  std::vector<double> hm((size_t)F * 6);
  for (int f = 0; f < F; ++f) {
    double th = 0.008 * std::sin(f * 0.7), c = std::cos(th), s = std::sin(th);
    double* m = &hm[(size_t)f * 6];
    m[0] = c; m[1] = -s; m[2] = 4 * std::sin(f * 1.3); m[3] = s; m[4] = c; m[5] = 4 * std::cos(f * 0.9);
  }
  CK(hipMalloc(&M, hm.size() * 8));
  CK(hipMemcpy(M, hm.data(), hm.size() * 8, hipMemcpyHostToDevice));
  const double gb = 2.0 * n * 2 / 1e9;
  auto report = [&](const char* name, float ms) {
    printf("%-44s %8.3f ms  %7.1f GB/s (algorithmic r+w)\n", name, ms, gb / (ms * 1e-3));
  };
  auto check = [&]() -> unsigned long long {
    (void)hipMemset(cnt, 0, 8);
    hipLaunchKernelGGL(diff_kernel, dim3(4096), dim3(256), 0, 0, dst, dst2, n, cnt);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost);
    return h;
  };
  void* ws;
  CK(hipMalloc(&ws, warp_workspace_bytes<WarpCfg<24, 8192, 6>>(F, H, W)));  // the most tiles
  using C32 = WarpCfg<32, 8192, 6>;
  using C40 = WarpCfg<40, 8192, 7>;
  using C48 = WarpCfg<48, 9216, 8>;
  using C56 = WarpCfg<56, 10240, 9>;
  using C64 = WarpCfg<64, 12288, 10>;
  // source values: 14-bit (exact integer blend everywhere), 13-bit with 0.1% hot pixels
  // (sparse float-faithful fallback, like the bench texture), full 16-bit (fallback in
  // nearly every row)
  std::vector<uint16_t> tex;
  if (argc > 2) {
    FILE* fp = fopen(argv[2], "rb");
    if (!fp) { printf("cannot open %s\n", argv[2]); return 1; }
    tex.resize((size_t)H * W);
    if (fread(tex.data(), 2, tex.size(), fp) != tex.size()) { printf("short texture file\n"); return 1; }
    fclose(fp);
  }
  const int only = getenv("LAB_DIST") ? atoi(getenv("LAB_DIST")) : -1;
  for (int dist = 0; dist < (tex.empty() ? 4 : 5); ++dist) {
    if (only >= 0 && dist != only) continue;
    static const char* dn[] = {"14-bit", "13-bit + 0.1% hot pixels", "16-bit", "13-bit + 1/8 of 32x32 blocks ~40k",
                               "bench texture (file)"};
    printf("-- source values: %s\n", dn[dist]);
    if (dist < 4) {
      hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, src, n, (uint32_t)dist);
    } else {
      CK(hipMemcpy(src, tex.data(), tex.size() * 2, hipMemcpyHostToDevice));
      for (int f = 1; f < F; ++f) CK(hipMemcpy(src + (size_t)f * H * W, src, tex.size() * 2, hipMemcpyDeviceToDevice));
    }
    if (getenv("LAB_GAP")) {  // kernel-boundary cost after a warp / after a copy (read with a kernel trace)
      unsigned* tp = reinterpret_cast<unsigned*>(cnt);
      hipEvent_t et, en;
      CK(hipEventCreate(&et));
      CK(hipEventCreateWithFlags(&en, hipEventDisableTiming));
      for (int k = 0; k < 4; ++k) {
        launch_warp<1>(src, dst, M, F, H, W, 0, ws, 0);
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, 0, tp);
        launch_warp<1>(src, dst, M, F, H, W, 0, ws, 0);
        CK(hipEventRecord(et, 0));  // a timing event between the warp and the next kernel
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, 0, tp);
        launch_warp<1>(src, dst, M, F, H, W, 0, ws, 0);
        CK(hipEventRecord(en, 0));  // a non-timing event
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, 0, tp);
        hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst2, n / 8);
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, 0, tp);
      }
      CK(hipDeviceSynchronize());
      continue;
    }
    if (getenv("LAB_LIB")) {  // the library's own configuration (BlockCfg), 3 repeats + output checksum
      for (int k = 0; k < 3; ++k)
        report("library cfg", timeit([&] { launch_warp<1>(src, dst, M, F, H, W, 0, ws, 0); }, reps));
      (void)hipMemset(cnt, 0, 8);
      hipLaunchKernelGGL(hash_kernel, dim3(4096), dim3(256), 0, 0, dst, n, cnt);
      unsigned long long h = 0;
      (void)hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost);
      printf("    output checksum %016llx\n", h);
      continue;
    }
    if (getenv("LAB_ONLY56")) {  // the library's configuration only, 3 repeats
      for (int k = 0; k < 3; ++k)
        report("128x56 (box 20 KB)", timeit([&] { launch_warp<1, C56>(src, dst, M, F, H, W, 0, ws, 0); }, reps));
      continue;
    }
    if (getenv("LAB_PITCH")) {  // fast-path tile heights that keep 7-8 workgroups per CU at kFastPitch
      using P40 = WarpCfg<40, 9216, 7>;
      using P48 = WarpCfg<48, 10240, 8>;
      using P56 = WarpCfg<56, 11672, 9>;
      printf("   kFastPitch %d\n", kFastPitch);
      for (int k = 0; k < 2; ++k) {
        report("128x56 (library cfg)", timeit([&] { launch_warp<1, C56>(src, dst, M, F, H, W, 0, ws, 0); }, reps));
        report("128x40 (18 KB)", timeit([&] { launch_warp<1, P40>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
        printf("    mismatches: %llu\n", check());
        report("128x48 (20 KB)", timeit([&] { launch_warp<1, P48>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
        printf("    mismatches: %llu\n", check());
        report("128x56 (22.8 KB)", timeit([&] { launch_warp<1, P56>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
        printf("    mismatches: %llu\n", check());
      }
      continue;
    }
    report("128x64 (box 24 KB)", timeit([&] { launch_warp<1, C64>(src, dst, M, F, H, W, 0, ws, 0); }, reps));
    report("128x32 (box 16 KB)", timeit([&] { launch_warp<1, C32>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
    printf("    mismatches vs 128x64: %llu\n", check());
    report("128x40 (box 16 KB)", timeit([&] { launch_warp<1, C40>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
    printf("    mismatches vs 128x64: %llu\n", check());
    report("128x48 (box 18 KB)", timeit([&] { launch_warp<1, C48>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
    printf("    mismatches vs 128x64: %llu\n", check());
    report("128x56 (box 20 KB)", timeit([&] { launch_warp<1, C56>(src, dst2, M, F, H, W, 0, ws, 0); }, reps));
    printf("    mismatches vs 128x64: %llu\n", check());
  }
  report("uint4 copy", timeit([&] {
    hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst2, n / 8); }, reps));
  CK(hipDeviceSynchronize());
  return 0;
}
