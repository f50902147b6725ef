// Memory-shape lab for the warp's HBM stream (not part of the library): copies of a
// 2000-frame 1080p u16 stack by tiles of TW x TH pixels, one 256-thread workgroup per
// tile, the way warp_affine_u16_kernel moves its bytes (16-byte loads of a tile's rows,
// stores of the same rows), against grid-stride copies.  Question: does the 256-byte row
// segment of a 128-pixel tile cost HBM efficiency against wider tiles?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/seg_lab.hip -o ab/seg_lab
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy_lin(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__global__ void copy_lin_nt(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + i), reinterpret_cast<u32x4*>(b) + i);
}

// one workgroup per TW x TH tile; W4 = store width (16: one uint4 per chunk, 4: the warp's
// one 4-byte word per lane, a wave = 256 B of a row); NT = nontemporal stores
template <int TW, int TH, int W4, bool NT>
__global__ __launch_bounds__(256) void copy_tile(const uint16_t* __restrict__ a, uint16_t* __restrict__ b, int H,
                                                 int W) {
  const int tiles_x = W / TW, tiles_y = (H + TH - 1) / TH;
  const int t = blockIdx.x;
  const int f = t / (tiles_x * tiles_y), r = t % (tiles_x * tiles_y);
  const int ty = r / tiles_x, tx = r % tiles_x;
  const size_t base = (size_t)f * H * W;
  constexpr int kChunks = TW / 8;  // 16-byte chunks per tile row
  constexpr int kPasses = (kChunks * TH + 255) / 256;
  uint4 v[kPasses];
#pragma unroll
  for (int k = 0; k < kPasses; ++k) {
    const int q = threadIdx.x + 256 * k, row = q / kChunks, c = q % kChunks;
    const int y = ty * TH + row;
    v[k] = make_uint4(0, 0, 0, 0);
    if (row < TH && y < H) v[k] = *reinterpret_cast<const uint4*>(a + base + (size_t)y * W + tx * TW + 8 * c);
  }
#pragma unroll
  for (int k = 0; k < kPasses; ++k) {
    const int q = threadIdx.x + 256 * k, row = q / kChunks, c = q % kChunks;
    const int y = ty * TH + row;
    if (row < TH && y < H) {
      uint16_t* d = b + base + (size_t)y * W + tx * TW + 8 * c;
      if (W4 == 16) {
        if (NT)
          __builtin_nontemporal_store(u32x4{v[k].x, v[k].y, v[k].z, v[k].w}, reinterpret_cast<u32x4*>(d));
        else
          *reinterpret_cast<uint4*>(d) = v[k];
      } else {  // four 4-byte stores per chunk (the warp stores one word per lane and row)
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (NT)
            __builtin_nontemporal_store(w[j], reinterpret_cast<uint32_t*>(d) + j);
          else
            reinterpret_cast<uint32_t*>(d)[j] = w[j];
        }
      }
    }
  }
}

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
  const int F = argc > 1 ? atoi(argv[1]) : 2000, reps = 10;
  const int H = argc > 3 ? atoi(argv[3]) : 1080, W = argc > 4 ? atoi(argv[4]) : 1920;
  const size_t n = (size_t)F * H * W;
  uint16_t *src, *dst;
  CK(hipMalloc(&src, n * 2));
  CK(hipMalloc(&dst, n * 2));
  CK(hipMemset(src, 1, n * 2));
  CK(hipMemset(dst, 0, n * 2));
  const double gb = 2.0 * n * 2 / 1e9;
  // a tile width that does not divide W copies only (W / TW) * TW columns: rates and the
  // full-frame-equivalent time count the bytes actually moved
  auto report = [&](const char* name, float ms, int TW = 0) {
    const double frac = TW ? (double)(W / TW * TW) / W : 1.0;
    printf("%-34s %.3f ms  %.2f TB/s  (full-frame equivalent %.3f ms)\n", name, ms, gb * frac / ms, ms / frac);
  };
  auto tiles = [&](int TW, int TH) { return F * (W / TW) * ((H + TH - 1) / TH); };
  const bool more = argc > 2 && argv[2][0] == 'm';
  const bool c3 = argc > 2 && argv[2][0] == 'c';
  for (int round = 0; round < 2; ++round) {
    report("linear uint4 copy", timeit([&] { hipLaunchKernelGGL(copy_lin, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n / 8); }, reps));
    report("linear uint4 copy, nt", timeit([&] { hipLaunchKernelGGL(copy_lin_nt, dim3(8192), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, n / 8); }, reps));
    report("tile 128x56, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 56, 4, true>), dim3(tiles(128, 56)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    report("tile 128x56, 16-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 56, 16, true>), dim3(tiles(128, 56)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    report("tile 128x56, 16-B stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 56, 16, false>), dim3(tiles(128, 56)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    report("tile 256x28, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 28, 4, true>), dim3(tiles(256, 28)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
    report("tile 256x28, 16-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 28, 16, true>), dim3(tiles(256, 28)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
    report("tile 640x12, 16-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<640, 12, 16, true>), dim3(tiles(640, 12)), dim3(256), 0, 0, src, dst, H, W); }, reps), 640);
    report("tile 1920x4, 16-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<1920, 4, 16, true>), dim3(tiles(1920, 4)), dim3(256), 0, 0, src, dst, H, W); }, reps), 1920);
    if (c3) {  // 512 x 512 frames: the warp's 128 x 64 tiles and others
      report("tile 128x64, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 64, 4, true>), dim3(tiles(128, 64)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
      report("tile 256x32, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 32, 4, true>), dim3(tiles(256, 32)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
      report("tile 512x16, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<512, 16, 4, true>), dim3(tiles(512, 16)), dim3(256), 0, 0, src, dst, H, W); }, reps), 512);
      report("tile 128x32, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 32, 4, true>), dim3(tiles(128, 32)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    }
    if (!more) continue;
    report("tile 128x28, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 28, 4, true>), dim3(tiles(128, 28)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    report("tile 128x112, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<128, 112, 4, true>), dim3(tiles(128, 112)), dim3(256), 0, 0, src, dst, H, W); }, reps), 128);
    report("tile 256x14, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 14, 4, true>), dim3(tiles(256, 14)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
    report("tile 256x56, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 56, 4, true>), dim3(tiles(256, 56)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
    report("tile 256x40, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<256, 40, 4, true>), dim3(tiles(256, 40)), dim3(256), 0, 0, src, dst, H, W); }, reps), 256);
    report("tile 384x20, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<384, 20, 4, true>), dim3(tiles(384, 20)), dim3(256), 0, 0, src, dst, H, W); }, reps), 384);
    report("tile 640x24, 4-B nt stores", timeit([&] { hipLaunchKernelGGL((copy_tile<640, 24, 4, true>), dim3(tiles(640, 24)), dim3(256), 0, 0, src, dst, H, W); }, reps), 640);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
