// K3: batched warpAffine of uint16 frames, OpenCV classic INTER_LINEAR semantics.
//
// Reference: VA:455-458  cv2.warpAffine(image, affine, image.shape[::-1],
// flags=cv2.INTER_LINEAR) -- no WARP_INVERSE_MAP, so OpenCV first inverts the 2x3
// map in double, then (WarpAffineInvoker) builds 1/32-pixel fixed-point source
// coordinates:  adelta[x] = cvRound(M0*x*1024), X0(y) = cvRound((M1*y + M2)*1024) + 16,
// X = (X0 + adelta[x]) >> 5, sx = X >> 5, fx = X & 31 (same for Y), and remapBilinear
// blends the four taps with float weights (1-fy/32, fy/32) x (1-fx/32, fx/32),
// ((v00*w0 + v01*w1) + v10*w2) + v11*w3 with separately rounded products, then
// cvRound to uint16 with saturation.  Taps outside the image read 0 (BORDER_CONSTANT).
// This file is compiled with -ffp-contract=off so that arithmetic is reproduced
// operation by operation.
//
// Layout: frames [F, H, W, C] u16 contiguous in HBM.  One workgroup covers a
// 128-column x 64-row output strip of one frame: the per-column deltas and per-row
// origins are computed once into LDS (the only double-precision work), then each
// thread produces 4 consecutive output pixels per row with integer coordinate
// arithmetic, gathers the taps through L1/L2 and writes one 8-byte store.
#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 128;  // output columns per workgroup (32 threads x 4 px)
constexpr int kTileH = 64;   // output rows per workgroup (8 row-groups x 8 passes)

__device__ __forceinline__ int cv_round(double v) { return (int)__builtin_rint(v); }

__device__ __forceinline__ uint16_t sat_u16(float v) {
  const int iv = (int)__builtin_rintf(v);
  return (uint16_t)((unsigned)iv <= 65535u ? iv : (iv > 0 ? 65535 : 0));
}

__device__ __forceinline__ int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// OpenCV warpAffine's in-place inversion of the forward map.
__device__ __forceinline__ void invert_affine(const double* Min, double* M) {
  for (int k = 0; k < 6; ++k) M[k] = Min[k];
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = M[4] * D, A22 = M[0] * D;
  M[0] = A11;
  M[1] *= -D;
  M[3] *= -D;
  M[4] = A22;
  const double b1 = -M[0] * M[2] - M[1] * M[5];
  const double b2 = -M[3] * M[2] - M[4] * M[5];
  M[2] = b1;
  M[5] = b2;
}

template <int C>
__device__ __forceinline__ void bilinear_px(const uint16_t* __restrict__ S, int H, int W, int X, int Y,
                                            uint16_t* out) {
  const int sx = sat_s16(X >> 5), sy = sat_s16(Y >> 5);
  const int fx = X & 31, fy = Y & 31;
  const float w0 = (float)((32 - fy) * (32 - fx)) * (1.f / 1024.f);
  const float w1 = (float)((32 - fy) * fx) * (1.f / 1024.f);
  const float w2 = (float)(fy * (32 - fx)) * (1.f / 1024.f);
  const float w3 = (float)(fy * fx) * (1.f / 1024.f);
  const bool x0 = (unsigned)sx < (unsigned)W, x1 = (unsigned)(sx + 1) < (unsigned)W;
  const bool y0 = (unsigned)sy < (unsigned)H, y1 = (unsigned)(sy + 1) < (unsigned)H;
  const size_t r0 = (size_t)sy * W, r1 = r0 + W;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const float v00 = (x0 && y0) ? (float)S[(r0 + sx) * C + k] : 0.f;
    const float v01 = (x1 && y0) ? (float)S[(r0 + sx + 1) * C + k] : 0.f;
    const float v10 = (x0 && y1) ? (float)S[(r1 + sx) * C + k] : 0.f;
    const float v11 = (x1 && y1) ? (float)S[(r1 + sx + 1) * C + k] : 0.f;
    out[k] = sat_u16(v00 * w0 + v01 * w1 + v10 * w2 + v11 * w3);
  }
}

template <int C>
__global__ __launch_bounds__(kThreads) void warp_affine_u16_kernel(const uint16_t* __restrict__ src,
                                                                   uint16_t* __restrict__ dst,
                                                                   const double* __restrict__ Mall, int H, int W,
                                                                   int inverse_map) {
  __shared__ int s_adelta[kTileW], s_bdelta[kTileW], s_X0[kTileH], s_Y0[kTileH];
  const int f = blockIdx.z;
  const int xb = blockIdx.x * kTileW, yb = blockIdx.y * kTileH;
  const int tid = threadIdx.x;
  double M[6];
  if (inverse_map) {
    for (int k = 0; k < 6; ++k) M[k] = Mall[6 * (size_t)f + k];
  } else {
    invert_affine(Mall + 6 * (size_t)f, M);
  }
  // per-column deltas (threads 0..127: a, 128..255: b) and per-row origins
  {
    const int x = xb + (tid & (kTileW - 1));
    if (tid < kTileW)
      s_adelta[tid] = cv_round(M[0] * x * 1024);
    else
      s_bdelta[tid - kTileW] = cv_round(M[3] * x * 1024);
    if (tid < 2 * kTileH) {
      const int y = yb + (tid & (kTileH - 1));
      if (tid < kTileH)
        s_X0[tid] = cv_round((M[1] * y + M[2]) * 1024) + 16;
      else
        s_Y0[tid - kTileH] = cv_round((M[4] * y + M[5]) * 1024) + 16;
    }
  }
  __syncthreads();
  const uint16_t* S = src + (size_t)f * H * W * C;
  uint16_t* Dst = dst + (size_t)f * H * W * C;
  const int tx = tid & 31, ty = tid >> 5;
  const int xl = tx * 4;
  const int x = xb + xl;
  int ad[4], bd[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    ad[p] = s_adelta[xl + p];
    bd[p] = s_bdelta[xl + p];
  }
  for (int rr = ty; rr < kTileH; rr += kThreads / 32) {
    const int y = yb + rr;
    if (y >= H) break;
    const int X0 = s_X0[rr], Y0 = s_Y0[rr];
    uint16_t o[4 * C];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int X = (X0 + ad[p]) >> 5, Y = (Y0 + bd[p]) >> 5;
      bilinear_px<C>(S, H, W, X, Y, o + p * C);
    }
    uint16_t* drow = Dst + ((size_t)y * W + x) * C;
    if (C == 1 && x + 4 <= W && (W & 3) == 0) {
      uint2 v;
      v.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
      v.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
      *reinterpret_cast<uint2*>(drow) = v;
    } else {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (x + p < W)
#pragma unroll
          for (int k = 0; k < C; ++k) drow[p * C + k] = o[p * C + k];
    }
  }
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_warp_affine_u16(kcmc_ctx* ctx, const uint16_t* src, uint16_t* dst, const double* M,
                                    int n_frames, int H, int W, int C, int inverse_map, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: ctx is NULL");
  if (n_frames < 0 || H < 0 || W < 0) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: negative size");
  if (n_frames == 0 || H == 0 || W == 0) return KCMC_OK;
  if (!src || !dst || !M) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: NULL pointer");
  if (H > 32767 || W > 32767) return fail(KCMC_EUNSUPPORTED, "kcmc_warp_affine_u16: H, W must be < 32768");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "kcmc_warp_affine_u16: at most 65535 frames per call");
  if (src == dst) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: in-place warp is not supported");
  dim3 grid(ceil_div(W, kTileW), ceil_div(H, kTileH), n_frames);
  hipStream_t s = (hipStream_t)stream;
  switch (C) {
    case 1:
      hipLaunchKernelGGL((warp_affine_u16_kernel<1>), grid, dim3(kThreads), 0, s, src, dst, M, H, W, inverse_map);
      break;
    case 3:
      hipLaunchKernelGGL((warp_affine_u16_kernel<3>), grid, dim3(kThreads), 0, s, src, dst, M, H, W, inverse_map);
      break;
    case 4:
      hipLaunchKernelGGL((warp_affine_u16_kernel<4>), grid, dim3(kThreads), 0, s, src, dst, M, H, W, inverse_map);
      break;
    default:
      return fail(KCMC_EUNSUPPORTED, "kcmc_warp_affine_u16: C must be 1, 3 or 4");
  }
  return launch_check("warp_affine_u16_kernel");
}
