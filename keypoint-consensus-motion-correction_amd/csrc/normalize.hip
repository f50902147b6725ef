// f2: the normalisation front end of align_images on the device (VA:100-104).
//
//   brightest = np.percentile(images, 99.99)                       (VA:102, VA:479-482)
//   images_u8 = np.clip(images / brightest * 255, 0, 255).astype(uint8)   (VA:484-492)
//
// Percentile: numpy's 'linear' method needs two order statistics of the flattened
// uint16 stack.  They are found exactly with two streaming passes of 256-bin
// histograms -- the high byte of every value, then the low byte of the values whose
// high byte is the coarse bin holding the wanted rank -- instead of a 65536-bin
// histogram (256 KB of counters does not fit one workgroup's LDS).  The host turns the
// counts into ranks and does numpy's interpolation in float64 (stages.py).
//
// Max-scale: every uint16 value maps to one uint8, so the host evaluates the reference's
// expression once per value (a 65536-entry table, bit-exact by construction) and the
// device applies it: LDS-resident table, 16 pixels per thread per step, 3 bytes of HBM
// traffic per pixel.
#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;

// bins[(v >> shift) & 255] over the values with (v >> 8) == match (match < 0: all).
// Video values crowd into a few coarse bins, so the LDS atomics must not collide: one
// sub-histogram per lane index (64 per workgroup, shared by the 4 waves, which issue their
// atomics at different times), rows padded to 257 words so that bin b of lane l sits in
// bank (l + b) % 64 -- the 64 atomics of one wave instruction hit 64 distinct banks
// whatever the values.  65.8 KB of LDS: two workgroups per CU.  The fine pass (match >= 0)
// counts only the values of one coarse bin -- few, for the 99.99th percentile -- and
// keeps 8 sub-histograms (8 KB) for occupancy instead.
constexpr int kRow = 257;

template <int R>
__global__ __launch_bounds__(kThreads) void hist256_u16_kernel(const uint16_t* __restrict__ src, size_t n, int shift,
                                                               int match, unsigned long long* __restrict__ out) {
  __shared__ uint32_t h[R * kRow];
  const int tid = threadIdx.x;
  for (int i = tid; i < R * kRow; i += kThreads) h[i] = 0u;
  __syncthreads();
  uint32_t* hl = h + (tid & (R - 1)) * kRow;
  const size_t n8 = n / 8;
  const uint4* s8 = reinterpret_cast<const uint4*>(src);
  const size_t stride = (size_t)gridDim.x * kThreads;
  auto count8 = [&](const uint4& q) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const uint32_t v = (w[k] >> (16 * p)) & 0xffffu;
        if (match < 0 || (int)(v >> 8) == match) atomicAdd(&hl[(v >> shift) & 255u], 1u);
      }
    }
  };
  size_t i = blockIdx.x * (size_t)kThreads + tid;
  for (; i + stride < n8; i += 2 * stride) {  // two 16-byte loads in flight per thread
    const uint4 a = s8[i], b = s8[i + stride];
    count8(a);
    count8(b);
  }
  if (i < n8) count8(s8[i]);
  if (blockIdx.x == 0) {  // tail (n % 8 values)
    for (size_t t = n8 * 8 + tid; t < n; t += kThreads) {
      const uint32_t v = src[t];
      if (match < 0 || (int)(v >> 8) == match) atomicAdd(&hl[(v >> shift) & 255u], 1u);
    }
  }
  __syncthreads();
  for (int b = tid; b < 256; b += kThreads) {
    unsigned long long c = 0;
    for (int r = 0; r < R; ++r) c += h[r * kRow + b];
    if (c) atomicAdd(&out[b], c);
  }
}

__global__ __launch_bounds__(kThreads) void lut_u16_to_u8_kernel(const uint16_t* __restrict__ src, size_t n,
                                                                 const uint8_t* __restrict__ lut,
                                                                 uint8_t* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) uint8_t t[65536];
  const int tid = threadIdx.x;
  for (int i = tid; i < 65536 / 16; i += kThreads)
    reinterpret_cast<uint4*>(t)[i] = reinterpret_cast<const uint4*>(lut)[i];
  __syncthreads();
  const size_t n16 = n / 16;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const size_t stride = (size_t)gridDim.x * kThreads;
  for (size_t i = blockIdx.x * (size_t)kThreads + tid; i < n16; i += stride) {
    const uint4 a = s[2 * i], b = s[2 * i + 1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = w[2 * k], hi = w[2 * k + 1];
      o[k] = (uint32_t)t[lo & 0xffffu] | ((uint32_t)t[lo >> 16] << 8) | ((uint32_t)t[hi & 0xffffu] << 16) |
             ((uint32_t)t[hi >> 16] << 24);
    }
    d[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  if (blockIdx.x == 0)
    for (size_t i = n16 * 16 + tid; i < n; i += kThreads) dst[i] = t[src[i]];
}

int grid_for(size_t work_items, size_t cap = 4096) {
  size_t g = (work_items + kThreads - 1) / kThreads;
  if (g > cap) g = cap;  // grid-stride beyond that
  return g < 1 ? 1 : (int)g;
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_histogram_u16(kcmc_ctx* ctx, const uint16_t* src, unsigned long long n, int shift, int match,
                                  unsigned long long* out_hist, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_histogram_u16: ctx is NULL");
  if (shift != 0 && shift != 8) return fail(KCMC_EINVAL, "kcmc_histogram_u16: shift must be 0 or 8");
  if (match > 255) return fail(KCMC_EINVAL, "kcmc_histogram_u16: match must be < 256");
  if (!out_hist || (n > 0 && !src)) return fail(KCMC_EINVAL, "kcmc_histogram_u16: NULL pointer");
  if (((uintptr_t)src & 15) != 0) return fail(KCMC_EINVAL, "kcmc_histogram_u16: src must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  KCMC_TRY(hip_check(hipMemsetAsync(out_hist, 0, 256 * sizeof(unsigned long long), s), "hipMemsetAsync"));
  if (n == 0) return KCMC_OK;
  if (match < 0)  // 2 resident workgroups per CU (LDS): a few waves of them
    hipLaunchKernelGGL(hist256_u16_kernel<64>, dim3(grid_for(n / 8 + 1, 2048)), dim3(kThreads), 0, s, src, (size_t)n,
                       shift, match, out_hist);
  else
    hipLaunchKernelGGL(hist256_u16_kernel<8>, dim3(grid_for(n / 8 + 1, 4096)), dim3(kThreads), 0, s, src, (size_t)n,
                       shift, match, out_hist);
  return launch_check("hist256_u16_kernel");
}

extern "C" int kcmc_lut_u16_to_u8(kcmc_ctx* ctx, const uint16_t* src, unsigned long long n, const uint8_t* lut,
                                  uint8_t* dst, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_lut_u16_to_u8: ctx is NULL");
  if (n == 0) return KCMC_OK;
  if (!src || !lut || !dst) return fail(KCMC_EINVAL, "kcmc_lut_u16_to_u8: NULL pointer");
  if ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)lut) & 15) != 0)
    return fail(KCMC_EINVAL, "kcmc_lut_u16_to_u8: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(lut_u16_to_u8_kernel, dim3(grid_for(n / 16 + 1)), dim3(kThreads), 0, (hipStream_t)stream, src,
                     (size_t)n, lut, dst);
  return launch_check("lut_u16_to_u8_kernel");
}
