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
constexpr int kTileW = 128;      // output columns per workgroup (32 threads x 2 pairs of pixels)
constexpr int kTileH = 64;       // output rows per workgroup (8 row groups x 8 passes)
constexpr int kLdsElems = 12288; // 24 KB of uint16 source staging per workgroup
constexpr int kMaxPitch = 256;   // staged row length limit (32 x 16-byte chunks)
constexpr int kRowPasses = 10;   // staging passes of 8 rows x 32 chunks: box rows <= 80

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

typedef float f2 __attribute__((ext_vector_type(2)));

// Bilinear blend of four taps exactly as remapBilinear<Cast<float, ushort>> does it:
// float weights tab[fy] x tab[fx] (each (32-f)/32 or f/32, products exact), separately
// rounded tap products, left-to-right sum.  Weight pairs use packed f32 math.
__device__ __forceinline__ uint16_t blend(float v00, float v01, float v10, float v11, int fx, int fy) {
  const f2 wx = __builtin_elementwise_fma(f2{(float)fx, (float)fx}, f2{-0.03125f, 0.03125f}, f2{1.f, 0.f});
  const f2 wy = __builtin_elementwise_fma(f2{(float)fy, (float)fy}, f2{-0.03125f, 0.03125f}, f2{1.f, 0.f});
  const f2 p01 = f2{v00, v01} * (wy.x * wx);
  const f2 p23 = f2{v10, v11} * (wy.y * wx);
  return sat_u16(((p01.x + p01.y) + p23.x) + p23.y);
}

// Direct-gather path (tiles whose source box does not fit the LDS budget): taps are
// loaded from clamped in-image addresses and zeroed when outside (branch-free, so the
// loads of a row's pixels are all in flight together).
template <int C>
__device__ __forceinline__ void bilinear_px(const uint16_t* __restrict__ S, int H, int W, int X, int Y,
                                            uint16_t* out) {
  const int sx = sat_s16(X >> 5), sy = sat_s16(Y >> 5);
  const int fx = X & 31, fy = Y & 31;
  const bool x0 = (unsigned)sx < (unsigned)W, x1 = (unsigned)(sx + 1) < (unsigned)W;
  const bool y0 = (unsigned)sy < (unsigned)H, y1 = (unsigned)(sy + 1) < (unsigned)H;
  const int cx0 = min(max(sx, 0), W - 1), cx1 = min(max(sx + 1, 0), W - 1);
  const int cy0 = min(max(sy, 0), H - 1), cy1 = min(max(sy + 1, 0), H - 1);
  const size_t r0 = (size_t)cy0 * W, r1 = (size_t)cy1 * W;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const uint16_t t00 = S[(r0 + cx0) * C + k], t01 = S[(r0 + cx1) * C + k];
    const uint16_t t10 = S[(r1 + cx0) * C + k], t11 = S[(r1 + cx1) * C + k];
    out[k] = blend((x0 && y0) ? (float)t00 : 0.f, (x1 && y0) ? (float)t01 : 0.f, (x0 && y1) ? (float)t10 : 0.f,
                   (x1 && y1) ? (float)t11 : 0.f, fx, fy);
  }
}

struct Box {
  int mode;   // 0: staged in LDS, 1: every tap outside the image (zeros), 2: direct gather
  int ax0;    // first staged column (multiple of 8)
  int sy0;    // first staged row
  int pitch;  // staged row length in pixels (multiple of 8)
  int rows;
};

// The source box of the tile's valid pixels.  adelta[x] = cvRound(M0*x*1024) and
// X0[y] = cvRound((M1*y + M2)*1024) + 16 are monotone in x and y (monotone products,
// sums and rounding), so their extremes sit at the tile's first/last valid column/row
// and sx = (X0[y] + adelta[x]) >> 10 spans [min, max] exactly; the second tap adds 1.
template <int C>
__device__ __forceinline__ Box source_box(const double* M, int xb, int yb, int H, int W) {
  const int xl = min(xb + kTileW, W) - 1, yl = min(yb + kTileH, H) - 1;
  const long long a0 = cv_round(M[0] * xb * 1024), a1 = cv_round(M[0] * xl * 1024);
  const long long b0 = cv_round(M[3] * xb * 1024), b1 = cv_round(M[3] * xl * 1024);
  const long long x0 = cv_round((M[1] * yb + M[2]) * 1024) + 16, x1 = cv_round((M[1] * yl + M[2]) * 1024) + 16;
  const long long y0 = cv_round((M[4] * yb + M[5]) * 1024) + 16, y1 = cv_round((M[4] * yl + M[5]) * 1024) + 16;
  const long long sx0 = (min(x0, x1) + min(a0, a1)) >> 10, sx1 = ((max(x0, x1) + max(a0, a1)) >> 10) + 1;
  const long long sy0 = (min(y0, y1) + min(b0, b1)) >> 10, sy1 = ((max(y0, y1) + max(b0, b1)) >> 10) + 1;
  Box b;
  const long long lim = 30000;  // keep clear of OpenCV's saturate_cast<short> on coordinates
  const bool small = sx0 > -lim && sx1 < lim && sy0 > -lim && sy1 < lim;
  const long long ax0 = (sx0 >> 3) << 3;
  const long long pitch = ((sx1 - ax0 + 1) + 7) & ~7ll;
  const long long rows = sy1 - sy0 + 1;
  b.mode = 2;
  if (small && (sx1 < 0 || sx0 > W - 1 || sy1 < 0 || sy0 > H - 1))
    b.mode = 1;
  else if (small && pitch <= kMaxPitch && rows <= 8 * kRowPasses && pitch * rows * C <= kLdsElems)
    b.mode = 0;
  b.ax0 = (int)ax0;
  b.sy0 = (int)sy0;
  b.pitch = (int)pitch;
  b.rows = (int)rows;
  return b;
}



// LDS tap read.  ALIGNED16 keeps every read a naturally aligned ds_read_u16 (the
// compiler otherwise fuses the two horizontal taps into one 4-byte read at a 2-byte
// aligned address).
template <bool ALIGNED16>
__device__ __forceinline__ float tap(const uint16_t* stile, int i) {
  if (ALIGNED16)
    return (float)__hip_atomic_load(const_cast<uint16_t*>(stile) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (float)stile[i];
}

// Output rows of one tile on one path (0: LDS-staged box, 1: zeros, 2: direct gather).
template <int C, int MODE, bool ALIGNED16 = false>
__device__ __forceinline__ void output_rows(const uint16_t* stile, const Box& box, const uint16_t* __restrict__ S,
                                            uint16_t* __restrict__ Dst, int H, int W, int xb, int yb, int tx, int ty,
                                            const int (&ad)[4], const int (&bd)[4], const int* s_X0,
                                            const int* s_Y0) {
  for (int rr = ty; rr < kTileH; rr += kThreads / 32) {
    const int y = yb + rr;
    if (y >= H) break;
    const int X0 = s_X0[rr], Y0 = s_Y0[rr];
    uint16_t o[4 * C];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int X = (X0 + ad[p]) >> 5, Y = (Y0 + bd[p]) >> 5;
      if (MODE == 0) {
        const int sx = X >> 5, sy = Y >> 5, fx = X & 31, fy = Y & 31;
        const int li = ((sy - box.sy0) * box.pitch + (sx - box.ax0)) * C;
#pragma unroll
        for (int k = 0; k < C; ++k) {
          const int i00 = li + k, i10 = li + box.pitch * C + k;
          o[p * C + k] = blend(tap<ALIGNED16>(stile, i00), tap<ALIGNED16>(stile, i00 + C), tap<ALIGNED16>(stile, i10),
                               tap<ALIGNED16>(stile, i10 + C), fx, fy);
        }
      } else if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < C; ++k) o[p * C + k] = 0;
      } else {
        bilinear_px<C>(S, H, W, X, Y, o + p * C);
      }
    }
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int x = xb + 2 * tx + 64 * pp;
      uint16_t* drow = Dst + ((size_t)y * W + x) * C;
      if (C == 1 && x + 2 <= W && (W & 1) == 0) {
        *reinterpret_cast<uint32_t*>(drow) = (uint32_t)o[2 * pp] | ((uint32_t)o[2 * pp + 1] << 16);
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (x + q < W)
#pragma unroll
            for (int k = 0; k < C; ++k) drow[q * C + k] = o[(2 * pp + q) * C + k];
      }
    }
  }
}

// VARIANT != 0 builds are ablations for tools/warp_lab.hip only (1: skip the per-pixel
// work, 2: skip the staging loads, 3: stores only, 4: aligned 16-bit tap reads); the
// library launches VARIANT 0.
template <int C, int VARIANT = 0>
__global__ __launch_bounds__(kThreads) void warp_affine_u16_kernel(const uint16_t* __restrict__ src,
                                                                   uint16_t* __restrict__ dst,
                                                                   const double* __restrict__ Mall, int H, int W,
                                                                   int inverse_map) {
  __shared__ __attribute__((aligned(16))) uint16_t stile[kLdsElems];
  __shared__ int s_adelta[kTileW], s_bdelta[kTileW], s_X0[kTileH], s_Y0[kTileH];
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so give each
  // XCD a contiguous run of tiles (neighbouring tiles share halo rows in that XCD's L2).
  const int ntx = gridDim.x, nty = gridDim.y;
  const int nwg = ntx * nty * gridDim.z;
  const int bid = blockIdx.x + ntx * (blockIdx.y + nty * blockIdx.z);
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int f = tile / (ntx * nty);
  const int t2 = tile - f * ntx * nty;
  const int xb = (t2 % ntx) * kTileW, yb = (t2 / ntx) * kTileH;
  const int tid = threadIdx.x;
  const uint16_t* S = src + (size_t)f * H * W * C;
  uint16_t* Dst = dst + (size_t)f * H * W * C;

  double M[6];
  if (inverse_map) {
    for (int k = 0; k < 6; ++k) M[k] = Mall[6 * (size_t)f + k];
  } else {
    invert_affine(Mall + 6 * (size_t)f, M);
  }
  const Box box = source_box<C>(M, xb, yb, H, W);
  const bool vec_stage = (C == 1) && ((W & 7) == 0);

  // ---- 1. issue the staging loads first (16-byte chunks; with W % 8 == 0 a chunk
  //         is either entirely inside the image or entirely outside -> zeros).
  //         Thread = (chunk c = tid & 31, row r = tid >> 5 + 8k): no integer division.
  uint4 chunk[kRowPasses];
  const int cpr = box.pitch >> 3;
  const int sc = tid & 31, sr = tid >> 5;
  const int gx = box.ax0 + 8 * sc;
  const bool col_ok = sc < cpr && gx >= 0 && gx < W;
  if (box.mode == 0 && vec_stage && VARIANT != 2 && VARIANT != 3) {
#pragma unroll
    for (int k = 0; k < kRowPasses; ++k) {
      const int r = sr + 8 * k;
      const int gy = box.sy0 + r;
      chunk[k] = make_uint4(0u, 0u, 0u, 0u);
      if (r < box.rows && col_ok && (unsigned)gy < (unsigned)H)
        chunk[k] = *reinterpret_cast<const uint4*>(S + (size_t)gy * W + gx);
    }
  }
  // ---- 2. fixed-point coordinate tables (WarpAffineInvoker), overlapping the loads
  {
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
  // ---- 3. land the staged box in LDS
  if (box.mode == 0) {
    if (vec_stage) {
#pragma unroll
      for (int k = 0; k < kRowPasses; ++k) {
        const int r = sr + 8 * k;
        if (r < box.rows && sc < cpr) *reinterpret_cast<uint4*>(&stile[r * box.pitch + 8 * sc]) = chunk[k];
      }
    } else {
      for (int q = tid; q < box.rows * box.pitch * C; q += kThreads) {
        const int r = q / (box.pitch * C), e = q - r * box.pitch * C;
        const int gy = box.sy0 + r, gx = box.ax0 + e / C, k = e % C;
        stile[q] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) ? S[((size_t)gy * W + gx) * C + k]
                                                                              : (uint16_t)0;
      }
    }
  }
  __syncthreads();

  // ---- 4. output: thread (tx, ty) makes pixel pairs x = xb + 2*tx + 64*pp (+0, +1)
  const int tx = tid & 31, ty = tid >> 5;
  // columns past the frame edge reuse the last valid column's coordinates so that
  // their (never stored) taps stay inside the staged box
  const int xlast = min(kTileW, W - xb) - 1;
  int ad[4], bd[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int xl = min(2 * tx + 64 * (p >> 1) + (p & 1), xlast);
    ad[p] = s_adelta[xl];
    bd[p] = s_bdelta[xl];
  }
  // one row loop per path (a path-uniform branch inside the loop would make the
  // compiler drain the previous rows' stores with s_waitcnt vmcnt(0) every row)
  if (VARIANT == 1 || VARIANT == 3)
    output_rows<C, 1>(stile, box, S, Dst, H, W, xb, yb, tx, ty, ad, bd, s_X0, s_Y0);
  else if (box.mode == 0 && VARIANT == 4)
    output_rows<C, 0, true>(stile, box, S, Dst, H, W, xb, yb, tx, ty, ad, bd, s_X0, s_Y0);
  else if (box.mode == 0)
    output_rows<C, 0>(stile, box, S, Dst, H, W, xb, yb, tx, ty, ad, bd, s_X0, s_Y0);
  else if (box.mode == 1)
    output_rows<C, 1>(stile, box, S, Dst, H, W, xb, yb, tx, ty, ad, bd, s_X0, s_Y0);
  else
    output_rows<C, 2>(stile, box, S, Dst, H, W, xb, yb, tx, ty, ad, bd, s_X0, s_Y0);
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
  if ((long long)grid.x * grid.y * grid.z >= (1ll << 31))
    return fail(KCMC_EUNSUPPORTED, "kcmc_warp_affine_u16: too many tiles in one call");
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
