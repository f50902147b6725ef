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
// 128-column x 32-row output tile of one frame.  The per-column deltas and per-row
// origins are computed once into LDS (the only double-precision work).  Because the
// fixed-point source coordinate is separable (X = X0[y] + adelta[x]), the exact source
// bounding box of the tile follows from four min/max reductions; the box is staged
// into LDS with coalesced 16-byte loads (zero outside the image, which is exactly
// BORDER_CONSTANT), and every output pixel gathers its four taps from LDS.  Each
// thread writes pixel pairs as 4-byte stores (a wave writes 256 contiguous bytes).
// Tiles whose box exceeds the 16 KB staging budget (strong zoom-out or rotation)
// gather from global memory instead; tiles whose box misses the image store zeros.
#include <climits>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 128;    // output columns per workgroup (32 threads x 2 pairs of pixels)
constexpr int kTileH = 32;     // output rows per workgroup (8 row groups x 4 passes)
constexpr int kLdsElems = 8192;  // 16 KB of uint16 source staging per workgroup

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

// Bilinear blend of four taps exactly as remapBilinear<Cast<float, ushort>> does it:
// float weights tab[fy] x tab[fx] (exact), separately rounded products, left-to-right sum.
__device__ __forceinline__ uint16_t blend(float v00, float v01, float v10, float v11, int fx, int fy) {
  const float wx0 = (float)(32 - fx) * 0.03125f, wx1 = (float)fx * 0.03125f;
  const float wy0 = (float)(32 - fy) * 0.03125f, wy1 = (float)fy * 0.03125f;
  return sat_u16(v00 * (wy0 * wx0) + v01 * (wy0 * wx1) + v10 * (wy1 * wx0) + v11 * (wy1 * wx1));
}

template <int C>
__global__ __launch_bounds__(kThreads) void warp_affine_u16_kernel(const uint16_t* __restrict__ src,
                                                                   uint16_t* __restrict__ dst,
                                                                   const double* __restrict__ Mall, int H, int W,
                                                                   int inverse_map) {
  __shared__ __attribute__((aligned(16))) uint16_t stile[kLdsElems];
  __shared__ int s_adelta[kTileW], s_bdelta[kTileW], s_X0[kTileH], s_Y0[kTileH];
  __shared__ int s_box[5];  // mode, ax0 (first staged column), sy0 (first staged row), pitch, rows
  const int f = blockIdx.z;
  const int xb = blockIdx.x * kTileW, yb = blockIdx.y * kTileH;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint16_t* S = src + (size_t)f * H * W * C;
  uint16_t* Dst = dst + (size_t)f * H * W * C;

  // ---- fixed-point coordinate tables (WarpAffineInvoker)
  {
    double M[6];
    if (inverse_map) {
      for (int k = 0; k < 6; ++k) M[k] = Mall[6 * (size_t)f + k];
    } else {
      invert_affine(Mall + 6 * (size_t)f, M);
    }
    const int xi = tid & (kTileW - 1);
    const int x = xb + xi;
    if (tid < kTileW)
      s_adelta[xi] = cv_round(M[0] * x * 1024);
    else
      s_bdelta[xi] = cv_round(M[3] * x * 1024);
    if (tid < 2 * kTileH) {
      const int yi = tid & (kTileH - 1);
      const int y = yb + yi;
      if (tid < kTileH)
        s_X0[yi] = cv_round((M[1] * y + M[2]) * 1024) + 16;
      else
        s_Y0[yi] = cv_round((M[4] * y + M[5]) * 1024) + 16;
    }
  }
  __syncthreads();
  // ---- exact source bounding box of the tile's valid pixels (wave 0)
  if (tid < 64) {
    int amin = INT_MAX, amax = INT_MIN, bmin = INT_MAX, bmax = INT_MIN;
    int xmin = INT_MAX, xmax = INT_MIN, ymin = INT_MAX, ymax = INT_MIN;
    for (int i = lane; i < kTileW; i += 64)
      if (xb + i < W) {
        amin = min(amin, s_adelta[i]);
        amax = max(amax, s_adelta[i]);
        bmin = min(bmin, s_bdelta[i]);
        bmax = max(bmax, s_bdelta[i]);
      }
    for (int i = lane; i < kTileH; i += 64)
      if (yb + i < H) {
        xmin = min(xmin, s_X0[i]);
        xmax = max(xmax, s_X0[i]);
        ymin = min(ymin, s_Y0[i]);
        ymax = max(ymax, s_Y0[i]);
      }
    for (int o = 32; o > 0; o >>= 1) {
      amin = min(amin, __shfl_xor(amin, o));
      amax = max(amax, __shfl_xor(amax, o));
      bmin = min(bmin, __shfl_xor(bmin, o));
      bmax = max(bmax, __shfl_xor(bmax, o));
      xmin = min(xmin, __shfl_xor(xmin, o));
      xmax = max(xmax, __shfl_xor(xmax, o));
      ymin = min(ymin, __shfl_xor(ymin, o));
      ymax = max(ymax, __shfl_xor(ymax, o));
    }
    if (lane == 0) {
      // sx = (X0 + adelta) >> 10; the second tap is sx + 1 (64-bit: no overflow here)
      const long long sx0 = ((long long)xmin + amin) >> 10, sx1 = (((long long)xmax + amax) >> 10) + 1;
      const long long sy0 = ((long long)ymin + bmin) >> 10, sy1 = (((long long)ymax + bmax) >> 10) + 1;
      int mode = 2;  // 0: staged in LDS, 1: all taps outside the image, 2: direct gather
      const long long lim = 30000;
      const bool small = sx0 > -lim && sx1 < lim && sy0 > -lim && sy1 < lim;
      if (small && (sx1 < 0 || sx0 > W - 1 || sy1 < 0 || sy0 > H - 1)) mode = 1;
      const long long ax0 = (sx0 >> 3) << 3;
      const long long pitch = ((sx1 - ax0 + 1) + 7) & ~7ll;
      const long long rows = sy1 - sy0 + 1;
      if (small && mode != 1 && pitch * rows * C <= kLdsElems) mode = 0;
      s_box[0] = mode;
      s_box[1] = (int)ax0;
      s_box[2] = (int)sy0;
      s_box[3] = (int)pitch;
      s_box[4] = (int)rows;
    }
  }
  __syncthreads();
  const int mode = s_box[0];
  const int ax0 = s_box[1], sy0 = s_box[2], pitch = s_box[3], rows = s_box[4];

  if (mode == 0) {
    // ---- stage the box (zeros outside the image)
    if (C == 1 && (W & 7) == 0) {
      const int cpr = pitch >> 3;  // 16-byte chunks per staged row
      for (int q = tid; q < rows * cpr; q += kThreads) {
        const int r = q / cpr, c = q - r * cpr;
        const int gy = sy0 + r, gx = ax0 + 8 * c;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if ((unsigned)gy < (unsigned)H) {
          const uint16_t* row = S + (size_t)gy * W;
          if (gx >= 0 && gx + 8 <= W) {
            v = *reinterpret_cast<const uint4*>(row + gx);
          } else {
            uint16_t e[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) e[k] = ((unsigned)(gx + k) < (unsigned)W) ? row[gx + k] : (uint16_t)0;
            v = make_uint4(e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
                           e[6] | ((uint32_t)e[7] << 16));
          }
        }
        *reinterpret_cast<uint4*>(&stile[r * pitch + 8 * c]) = v;
      }
    } else {
      for (int q = tid; q < rows * pitch * C; q += kThreads) {
        const int r = q / (pitch * C), e = q - r * pitch * C;
        const int gy = sy0 + r, gx = ax0 + e / C, k = e % C;
        stile[q] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) ? S[((size_t)gy * W + gx) * C + k]
                                                                              : (uint16_t)0;
      }
    }
    __syncthreads();
  }

  // ---- output: thread (tx, ty) makes pixel pairs x = xb + 2*tx + 64*pp (+0, +1)
  const int tx = tid & 31, ty = tid >> 5;
  for (int rr = ty; rr < kTileH; rr += kThreads / 32) {
    const int y = yb + rr;
    if (y >= H) break;
    const int X0 = s_X0[rr], Y0 = s_Y0[rr];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int xl = 2 * tx + 64 * pp;
      const int x = xb + xl;
      uint16_t o[2 * C];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int X = (X0 + s_adelta[xl + q]) >> 5, Y = (Y0 + s_bdelta[xl + q]) >> 5;
        if (x + q >= W) {  // outside the frame: nothing to compute or store
#pragma unroll
          for (int k = 0; k < C; ++k) o[q * C + k] = 0;
        } else if (mode == 0) {
          const int sx = X >> 5, sy = Y >> 5, fx = X & 31, fy = Y & 31;
          const int li = ((sy - sy0) * pitch + (sx - ax0)) * C;
#pragma unroll
          for (int k = 0; k < C; ++k)
            o[q * C + k] = blend((float)stile[li + k], (float)stile[li + C + k], (float)stile[li + pitch * C + k],
                                 (float)stile[li + pitch * C + C + k], fx, fy);
        } else if (mode == 1) {
#pragma unroll
          for (int k = 0; k < C; ++k) o[q * C + k] = 0;
        } else {
          bilinear_px<C>(S, H, W, X, Y, o + q * C);
        }
      }
      uint16_t* drow = Dst + ((size_t)y * W + x) * C;
      if (C == 1 && x + 2 <= W && (W & 1) == 0) {
        *reinterpret_cast<uint32_t*>(drow) = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (x + q < W)
#pragma unroll
            for (int k = 0; k < C; ++k) drow[q * C + k] = o[q * C + k];
      }
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
