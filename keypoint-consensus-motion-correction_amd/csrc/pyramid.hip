// f4: the spatial downsample of VideoAligner._downsample (VA:494-506) on the device:
// cv2.pyrDown(frame, dstsize) of every uint8 sample frame, OpenCV's pyrDown_ semantics
// (imgproc/src/pyramids.cpp):
//
//   dst(x, y) = (sum_{i,j} k_i k_j src(r(2y + i - 2), r(2x + j - 2)) + 128) >> 8,
//   k = (1, 4, 6, 4, 1),  r = borderInterpolate(., BORDER_REFLECT_101)
//
// (the ring-buffer row pass, its tabL/tabR border columns and FixPtCast<uchar, 8> give
// exactly this integer expression; every intermediate fits 16 bits, the total <= 65280).
// dstsize must satisfy OpenCV's assertion |2 dst_w - W| <= 2, |2 dst_h - H| <= 2.
//
// One workgroup per 64 x 32 output tile: the (68 x 136)-byte source window is staged
// into LDS with 4-byte loads (reflected bytes at the frame border), the horizontal pass
// makes four column sums per v_dot4_u32_u8 step (weights 1,4,6,4 packed, the fifth tap
// as the accumulator), and the vertical pass runs on packed 16-bit pairs before four
// output bytes are stored as one word.  HBM-bound: 1.25 bytes per source pixel.
#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 64;                 // output columns per tile
constexpr int kTileH = 32;                 // output rows per tile
constexpr int kSrcRows = 2 * kTileH + 4;   // 68 staged source rows
constexpr int kSrcCols = 2 * kTileW + 8;   // 136 staged bytes per row (from 2 x0 - 4)
constexpr int kSrcWords = kSrcCols / 4;    // 34

__device__ __forceinline__ int reflect101(int p, int len) {
  if (len == 1) return 0;
  while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
  return p;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(kThreads) void pyr_down_u8_kernel(const uint8_t* __restrict__ src,
                                                               uint8_t* __restrict__ dst, int H, int W, int DH,
                                                               int DW) {
  __shared__ __attribute__((aligned(16))) uint32_t s[kSrcRows * kSrcWords];  // bytes [r][136]
  __shared__ __attribute__((aligned(16))) uint16_t hs[kSrcRows * kTileW];   // row sums [r][64]
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTileH;
  const uint8_t* S = src + (size_t)blockIdx.z * H * W;
  uint8_t* D = dst + (size_t)blockIdx.z * DH * DW;

  // stage source rows 2 y0 - 2 + r, bytes 2 x0 - 4 + c (reflected at the border)
  const bool words = (W & 3) == 0;
  for (int q = tid; q < kSrcRows * kSrcWords; q += kThreads) {
    const int r = q / kSrcWords, w = q - r * kSrcWords;
    const int gy = reflect101(2 * y0 - 2 + r, H);
    const int gx = 2 * x0 - 4 + 4 * w;
    const uint8_t* row = S + (size_t)gy * W;
    uint32_t v;
    if (words && gx >= 0 && gx + 4 <= W) {
      v = *reinterpret_cast<const uint32_t*>(row + gx);
    } else {
      v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= (uint32_t)row[reflect101(gx + b, W)] << (8 * b);
    }
    s[q] = v;
  }
  __syncthreads();

  // horizontal pass: hs[r][c] = sum_j k_j src[r][2c + j] (staged bytes 2c + 2 .. 2c + 6);
  // a work item is 4 output columns 4g .. 4g + 3 = staged words 2g .. 2g + 3
  for (int q = tid; q < kSrcRows * (kTileW / 4); q += kThreads) {
    const int r = q >> 4, g = q & 15;
    const uint32_t* w = s + r * kSrcWords + 2 * g;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
    const uint32_t k = 0x04060401u;  // bytes (1, 4, 6, 4)
    const uint32_t h0 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbit(w1, w0, 16), k, (w1 >> 16) & 255u, false);
    const uint32_t h1 = __builtin_amdgcn_udot4(w1, k, w2 & 255u, false);
    const uint32_t h2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbit(w2, w1, 16), k, (w2 >> 16) & 255u, false);
    const uint32_t h3 = __builtin_amdgcn_udot4(w2, k, w3 & 255u, false);
    uint2 out;
    out.x = h0 | (h1 << 16);
    out.y = h2 | (h3 << 16);
    *reinterpret_cast<uint2*>(hs + r * kTileW + 4 * g) = out;
  }
  __syncthreads();

  // vertical pass on packed 16-bit pairs: (h0 + 4 h1 + 6 h2 + 4 h3 + h4 + 128) >> 8
  for (int q = tid; q < kTileH * (kTileW / 4); q += kThreads) {
    const int j = q >> 4, g = q & 15;
    const int y = y0 + j, x = x0 + 4 * g;
    if (y >= DH || x >= DW) continue;
    u16x2 lo = {128, 128}, hi = {128, 128};
    const u16x2 wt[5] = {{1, 1}, {4, 4}, {6, 6}, {4, 4}, {1, 1}};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint2 p = *reinterpret_cast<const uint2*>(hs + (2 * j + i) * kTileW + 4 * g);
      lo += __builtin_bit_cast(u16x2, p.x) * wt[i];
      hi += __builtin_bit_cast(u16x2, p.y) * wt[i];
    }
    lo >>= 8;
    hi >>= 8;
    const uint32_t packed = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo),
                                                  0x06040200u);
    uint8_t* drow = D + (size_t)y * DW + x;
    if ((DW & 3) == 0) {  // x + 4 <= DW, aligned
      *reinterpret_cast<uint32_t*>(drow) = packed;
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (x + b < DW) drow[b] = (uint8_t)(packed >> (8 * b));
    }
  }
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_pyr_down_u8(kcmc_ctx* ctx, const uint8_t* src, int n_frames, int H, int W, uint8_t* dst,
                                int dst_h, int dst_w, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_pyr_down_u8: ctx is NULL");
  if (n_frames < 0) return fail(KCMC_EINVAL, "kcmc_pyr_down_u8: negative frame count");
  if (H <= 0 || W <= 0) return fail(KCMC_EINVAL, "kcmc_pyr_down_u8: ssize.width > 0 && ssize.height > 0 violated");
  if (dst_w <= 0 || dst_h <= 0 || std::abs(dst_w * 2 - W) > 2 || std::abs(dst_h * 2 - H) > 2)
    return fail(KCMC_EINVAL,
                "kcmc_pyr_down_u8: std::abs(dsize.width*2 - ssize.width) <= 2 && "
                "std::abs(dsize.height*2 - ssize.height) <= 2 violated");
  if (n_frames == 0) return KCMC_OK;
  if (!src || !dst) return fail(KCMC_EINVAL, "kcmc_pyr_down_u8: NULL pointer");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "kcmc_pyr_down_u8: at most 65535 frames per call");
  if (((uintptr_t)src | (uintptr_t)dst) & 3) return fail(KCMC_EINVAL, "kcmc_pyr_down_u8: buffers must be 4-byte aligned");
  hipLaunchKernelGGL(pyr_down_u8_kernel, dim3(ceil_div(dst_w, kTileW), ceil_div(dst_h, kTileH), n_frames),
                     dim3(kThreads), 0, (hipStream_t)stream, src, dst, H, W, dst_h, dst_w);
  return launch_check("pyr_down_u8_kernel");
}
