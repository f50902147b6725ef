// HBM bandwidth lab (not part of the library): what a streaming copy of the warp's
// footprint (2000 x 1080p u16 = 8.29 GB read + 8.29 GB written) reaches on this box
// with different load/store shapes.  Build here:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bw_lab.hip -o tools/bw_lab
// Run on the GPU box: tools/bw_lab [GB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      printf("%s: %s\n", #x, hipGetErrorString(e));                      \
      return 1;                                                          \
    }                                                                    \
  } while (0)

__global__ void copy_gs(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// U uint4 per thread per step, all loads issued before the stores.
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_unroll(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * blockDim.x;
      if (i < n) {
        if (NT) {
          const uint32_t* p = reinterpret_cast<const uint32_t*>(a + i);
          v[u] = make_uint4(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                            __builtin_nontemporal_load(p + 2), __builtin_nontemporal_load(p + 3));
        } else {
          v[u] = a[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * blockDim.x;
      if (i < n) {
        if (NT) {
          uint32_t* p = reinterpret_cast<uint32_t*>(b + i);
          __builtin_nontemporal_store(v[u].x, p);
          __builtin_nontemporal_store(v[u].y, p + 1);
          __builtin_nontemporal_store(v[u].z, p + 2);
          __builtin_nontemporal_store(v[u].w, p + 3);
        } else
          b[i] = v[u];
      }
    }
  }
}

// One workgroup per contiguous chunk (like one warp tile per workgroup), no grid-stride.
template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + (size_t)u * blockDim.x;
    if (i < n) v[u] = a[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + (size_t)u * blockDim.x;
    if (i < n) b[i] = v[u];
  }
}

__global__ void read_only(const uint4* __restrict__ a, size_t n, unsigned* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void write_only(uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
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
  const double gb = argc > 1 ? atof(argv[1]) : 8.2944;  // one direction
  const size_t n = (size_t)(gb * 1e9 / 16);
  uint4 *a, *b;
  unsigned* o;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&o, 16));
  CK(hipMemset(a, 1, n * 16));
  CK(hipMemset(b, 0, n * 16));
  const double bytes2 = 2.0 * n * 16;
  const int reps = 5;
  auto report = [&](const char* name, float ms, double bytes) {
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy grid-stride x1 (grid %d)", g);
    report(nm, timeit([&] { hipLaunchKernelGGL(copy_gs, dim3(g), dim3(256), 0, 0, a, b, n); }, reps), bytes2);
  }
  for (int g : {2048, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy unroll4 (grid %d)", g);
    report(nm, timeit([&] { hipLaunchKernelGGL((copy_unroll<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps),
           bytes2);
    snprintf(nm, sizeof nm, "copy unroll4 nontemporal (grid %d)", g);
    report(nm, timeit([&] { hipLaunchKernelGGL((copy_unroll<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps),
           bytes2);
    snprintf(nm, sizeof nm, "copy unroll8 (grid %d)", g);
    report(nm, timeit([&] { hipLaunchKernelGGL((copy_unroll<8, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, reps),
           bytes2);
  }
  {
    const unsigned g4 = (unsigned)((n + 256 * 4 - 1) / (256 * 4));
    report("copy chunk x4 (1 chunk/WG)",
           timeit([&] { hipLaunchKernelGGL((copy_chunk<4>), dim3(g4), dim3(256), 0, 0, a, b, n); }, reps), bytes2);
    const unsigned g8 = (unsigned)((n + 256 * 8 - 1) / (256 * 8));
    report("copy chunk x8 (1 chunk/WG)",
           timeit([&] { hipLaunchKernelGGL((copy_chunk<8>), dim3(g8), dim3(256), 0, 0, a, b, n); }, reps), bytes2);
  }
  report("read only (grid 4096)", timeit([&] { hipLaunchKernelGGL(read_only, dim3(4096), dim3(256), 0, 0, a, n, o); }, reps),
         n * 16.0);
  report("write only (grid 4096)", timeit([&] { hipLaunchKernelGGL(write_only, dim3(4096), dim3(256), 0, 0, b, n); }, reps),
         n * 16.0);
  CK(hipDeviceSynchronize());
  return 0;
}
