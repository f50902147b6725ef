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
// One thread per 4 output columns x 16 output rows, no LDS: the thread walks down its
// strip keeping the horizontal sums of the last five source rows in registers (two new
// source rows per output row, each one 16-byte load covering the 11 bytes its 4 outputs
// need), makes four column sums per v_dot4_u32_u8 (weights 1,4,6,4 packed, the fifth tap
// as the accumulator), runs the vertical pass on packed 16-bit pairs and stores the four
// output bytes as one word.  Lanes whose window crosses the frame edge (or frames with
// W % 4 != 0) gather reflected bytes one by one.  HBM-bound: 1.25 bytes per source px.
#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kGroupsX = 64;   // threads along x per workgroup (4 output columns each)
constexpr int kStripsY = 4;    // threads along y per workgroup
constexpr int kStripH = 16;    // output rows per thread

__device__ __forceinline__ int reflect101(int p, int len) {
  if (len == 1) return 0;
  while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
  return p;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Horizontal 1-4-6-4-1 sums of one source row for the outputs x .. x + 3 (source bytes
// 2x - 2 .. 2x + 8), packed as (h0 | h1 << 16, h2 | h3 << 16).
struct HRow {
  uint32_t a, b;
};

__device__ __forceinline__ HRow hsums(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  // w0..w3 = source bytes 2x - 4 .. 2x + 11; output x + k needs bytes 2x - 2 + 2k .. 2x + 2 + 2k
  const uint32_t k = 0x04060401u;  // bytes (1, 4, 6, 4)
  const uint32_t h0 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbit(w1, w0, 16), k, (w1 >> 16) & 255u, false);
  const uint32_t h1 = __builtin_amdgcn_udot4(w1, k, w2 & 255u, false);
  const uint32_t h2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbit(w2, w1, 16), k, (w2 >> 16) & 255u, false);
  const uint32_t h3 = __builtin_amdgcn_udot4(w2, k, w3 & 255u, false);
  return HRow{h0 | (h1 << 16), h2 | (h3 << 16)};
}

// Source bytes 2x - 4 .. 2x + 11 of one row (the fast path: one 16-byte load; at the
// frame edge the 11 needed bytes one by one, reflected).
__device__ __forceinline__ uint4 load_row(const uint8_t* __restrict__ row, int x, int W, bool fast) {
  if (fast) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(row + 2 * x - 4);
    return make_uint4(p[0], p[1], p[2], p[3]);
  }
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = 2 * x - 4 + 4 * i + b;
      if (c >= 2 * x - 2 && c <= 2 * x + 8) w[i] |= (uint32_t)row[reflect101(c, W)] << (8 * b);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ HRow hrow(const uint4& w) { return hsums(w.x, w.y, w.z, w.w); }

// The thread's strip: output rows y0 .. y1 - 1 of columns x .. x + 3, software-pipelined
// one output row ahead (the two source rows of row y + 1 are loaded before row y is
// blended).  Every load is in bounds: rows are reflected.  (Fully unrolled strips, or
// separate fast/edge instantiations, measured 20-25 % slower: more VGPRs, lower occupancy.)
__device__ __forceinline__ void strip(const uint8_t* __restrict__ S, uint8_t* __restrict__ D, int H, int W, int DW,
                                      int x, int y0, int y1, bool fast) {
  HRow r0 = hrow(load_row(S + (size_t)reflect101(2 * y0 - 2, H) * W, x, W, fast));
  HRow r1 = hrow(load_row(S + (size_t)reflect101(2 * y0 - 1, H) * W, x, W, fast));
  HRow r2 = hrow(load_row(S + (size_t)reflect101(2 * y0, H) * W, x, W, fast));
  HRow r3 = hrow(load_row(S + (size_t)reflect101(2 * y0 + 1, H) * W, x, W, fast));
  HRow r4 = hrow(load_row(S + (size_t)reflect101(2 * y0 + 2, H) * W, x, W, fast));
  uint4 n3 = load_row(S + (size_t)reflect101(2 * y0 + 3, H) * W, x, W, fast);
  uint4 n4 = load_row(S + (size_t)reflect101(2 * y0 + 4, H) * W, x, W, fast);
  const u16x2 c4 = {4, 4}, c6 = {6, 6}, c128 = {128, 128};
  for (int y = y0; y < y1; ++y) {
    if (y > y0) {
      r0 = r2;
      r1 = r3;
      r2 = r4;
      r3 = hrow(n3);
      r4 = hrow(n4);
      n3 = load_row(S + (size_t)reflect101(2 * y + 3, H) * W, x, W, fast);
      n4 = load_row(S + (size_t)reflect101(2 * y + 4, H) * W, x, W, fast);
    }
    // (h0 + 4 h1 + 6 h2 + 4 h3 + h4 + 128) >> 8 on packed 16-bit pairs (<= 65408)
    u16x2 lo = __builtin_bit_cast(u16x2, r0.a) + __builtin_bit_cast(u16x2, r4.a) + c128 +
               c4 * (__builtin_bit_cast(u16x2, r1.a) + __builtin_bit_cast(u16x2, r3.a)) +
               c6 * __builtin_bit_cast(u16x2, r2.a);
    u16x2 hi = __builtin_bit_cast(u16x2, r0.b) + __builtin_bit_cast(u16x2, r4.b) + c128 +
               c4 * (__builtin_bit_cast(u16x2, r1.b) + __builtin_bit_cast(u16x2, r3.b)) +
               c6 * __builtin_bit_cast(u16x2, r2.b);
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

__global__ __launch_bounds__(kGroupsX * kStripsY) void pyr_down_u8_kernel(const uint8_t* __restrict__ src,
                                                                         uint8_t* __restrict__ dst, int H, int W,
                                                                         int DH, int DW) {
  const int x = 4 * (blockIdx.x * kGroupsX + threadIdx.x);
  const int y0 = kStripH * (blockIdx.y * kStripsY + threadIdx.y);
  if (x >= DW || y0 >= DH) return;  // no barriers below
  const int y1 = min(y0 + kStripH, DH);
  const uint8_t* S = src + (size_t)blockIdx.z * H * W;
  uint8_t* D = dst + (size_t)blockIdx.z * DH * DW;
  strip(S, D, H, W, DW, x, y0, y1, (W & 3) == 0 && 2 * x - 4 >= 0 && 2 * x + 12 <= W);
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
  hipLaunchKernelGGL(pyr_down_u8_kernel,
                     dim3(ceil_div(ceil_div(dst_w, 4), kGroupsX), ceil_div(ceil_div(dst_h, kStripH), kStripsY), n_frames),
                     dim3(kGroupsX, kStripsY), 0, (hipStream_t)stream, src, dst, H, W, dst_h, dst_w);
  return launch_check("pyr_down_u8_kernel");
}
