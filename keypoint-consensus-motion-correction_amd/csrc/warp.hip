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
// Layout: frames [F, H, W, C] u16 contiguous in HBM, processed in 128 x 56 output
// tiles.  Because the fixed-point source coordinate is separable (X = X0[y] + adelta[x])
// and monotone, the exact source bounding box of a tile follows from its corner values;
// the box is staged into LDS with coalesced 16-byte loads (zero outside the image,
// which is exactly BORDER_CONSTANT) and every output pixel gathers its four taps from
// LDS with aligned 16-bit reads.  A wave makes one 128-pixel output row at a time
// (lane l: pixels 2l, 2l+1, one 4-byte store), so its tap reads cover consecutive LDS
// words without bank conflicts and its row-level state is wave-uniform.  Tiles whose box exceeds the staging budget (strong
// zoom-out or rotation) gather from global memory instead; tiles whose box misses the
// image store zeros.
//
// One-channel frames with W % 8 == 0 and a box that fits a fixed 144-pixel LDS pitch (the
// near-identity maps of motion correction) take a leaner form of the same path (mode 3,
// fast_rows): scalar per-row origins from a per-frame table, immediate-offset taps, buffer
// stores, and a per-tile choice of blend from the staged values (exact integer blend with
// no range check when every value is < 16384; OpenCV's float blend on packed fp32 for
// bright boxes).
//
// Two launches: warp_plan_kernel (one thread per tile) inverts the map in fp64 and
// derives each tile's source box and the frame's row-origin table, so that the tile
// kernel starts with scalar loads of its plan and issues its staging loads immediately; warp_affine_u16_kernel then makes
// one tile per workgroup, latency hidden by the other resident workgroups (a persistent
// double-buffered variant measured 25% slower).
#include <climits>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;
constexpr int kTileW = 128;     // output columns per tile (64 lanes x 2 pixels)
constexpr int kMaxPitch = 256;  // staged row length limit (32 x 16-byte chunks)

template <int TILE_H, int LDS_ELEMS, int ROW_PASSES>
struct WarpCfg {
  static constexpr int kTileH = TILE_H;          // output rows per tile (4 waves x kTileH/4)
  static constexpr int kLdsElems = LDS_ELEMS;    // uint16 staging budget per box
  static constexpr int kRowPasses = ROW_PASSES;  // staging passes of 8 rows x 32 chunks
};
using BlockCfg = WarpCfg<56, 10240, 9>;  // 20 KB box, box rows <= 72 (7 workgroups per CU)
// Frame heights that are a multiple of 64 but not of 56 (512: config 3) lose 9 % of their
// tiles to a partial last tile row at 56 rows; 64-row tiles with the same 20 KB box budget
// cover them exactly (the fast path's 71 staged rows still hold a 64-row tile rotated by up
// to ~2.5 deg; larger rotations take the general staged path or the direct gather).
using Block64Cfg = WarpCfg<64, 10240, 9>;

// one-channel tile height for a frame height (round 3)
inline bool use_tile64(int H) { return H % 64 == 0 && H % 56 != 0; }
// Multi-channel frames (RGB / RGBA, config 4): 3-4x the bytes per box pixel, so shorter
// tiles keep the interleaved box in a 32 KB LDS budget (box rows <= 32).
using ChanCfg = WarpCfg<24, 16384, 4>;

template <int C>
struct CfgFor {
  using type = BlockCfg;
};
template <>
struct CfgFor<3> {
  using type = ChanCfg;
};
template <>
struct CfgFor<4> {
  using type = ChanCfg;
};

// Fast staged path (mode 3; one channel, W % 8 == 0, the near-identity maps of motion
// correction): the box is staged at a fixed LDS pitch, so the lower tap row is an
// immediate offset of the upper one, and the per-row source origins come from a per-frame
// table through scalar loads.  Boxes wider than kFastPitch or taller than kFastRows take
// the general staged path (mode 0).
constexpr int kFastPitch = 144;  // pixels: 128-px tile + up to ~8 deg / 6 % zoom
constexpr int kFastChunks = kFastPitch / 8;  // 16-byte chunks per staged row
template <class Cfg>
struct Fast {
  static constexpr int kRows = (Cfg::kLdsElems - 8) / kFastPitch;  // the last 16 bytes: per-wave flags
  static constexpr int kFlagWord = Cfg::kLdsElems / 2 - 4;          // uint32 index of the flags
  static constexpr int kPasses = (kRows * kFastChunks + kThreads - 1) / kThreads;
};

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

// Frames whose map holds a NaN (no RANSAC model) are warped to zeros, as OpenCV's
// BORDER_CONSTANT gives for coordinates that land outside the image; the pipeline warps
// them again with the gap-filled maps (VA:347-407) before handing the frames out.
__device__ __forceinline__ bool map_has_nan(const double* M, int n) {
  bool nan = false;
  for (int k = 0; k < n; ++k) nan = nan || M[k] != M[k];
  return nan;
}

__device__ __forceinline__ void load_map(const double* __restrict__ Mall, int f, int inverse_map, double* M) {
  if (inverse_map) {
    for (int k = 0; k < 6; ++k) M[k] = Mall[6 * (size_t)f + k];
  } else {
    invert_affine(Mall + 6 * (size_t)f, M);
  }
}

// remapBilinear<Cast<float, ushort>>'s blend in exact integer/float steps that are cheap
// on the VALU: w_k = K_k / 1024 with K_k = (32-fy|fy) * (32-fx|fx) an integer, and
// fl(v * K/1024) = fl(v*K) * 2^-10 (power-of-two scaling commutes with rounding), where
// fl(v*K) = cvt_f32_u32(v*K) because the integer product is exact and the conversion
// rounds to nearest-even like the multiply.  The left-to-right sum scales the same way.
__device__ __forceinline__ uint16_t blend_int(uint32_t v00, uint32_t v01, uint32_t v10, uint32_t v11, int fx,
                                              int fy) {
  const uint32_t ax = 32 - fx, ay = 32 - fy;
  const float q0 = (float)__umul24(v00, __umul24(ay, ax));
  const float q1 = (float)__umul24(v01, __umul24(ay, (uint32_t)fx));
  const float q2 = (float)__umul24(v10, __umul24((uint32_t)fy, ax));
  const float q3 = (float)__umul24(v11, __umul24((uint32_t)fy, (uint32_t)fx));
  return sat_u16((((q0 + q1) + q2) + q3) * 0.0009765625f);
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
    const uint32_t t00 = S[(r0 + cx0) * C + k], t01 = S[(r0 + cx1) * C + k];
    const uint32_t t10 = S[(r1 + cx0) * C + k], t11 = S[(r1 + cx1) * C + k];
    out[k] = blend_int((x0 && y0) ? t00 : 0u, (x1 && y0) ? t01 : 0u, (x0 && y1) ? t10 : 0u, (x1 && y1) ? t11 : 0u,
                       fx, fy);
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
template <class Cfg, int C>
__device__ __forceinline__ Box source_box(const double* M, int xb, int yb, int H, int W) {
  const int xl = min(xb + kTileW, W) - 1, yl = min(yb + Cfg::kTileH, H) - 1;
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
  else if (small && pitch <= kMaxPitch && rows <= 8 * Cfg::kRowPasses && pitch * rows * C <= Cfg::kLdsElems)
    b.mode = 0;
  b.ax0 = (int)ax0;
  b.sy0 = (int)sy0;
  b.pitch = (int)pitch;
  b.rows = (int)rows;
  return b;
}

// Staging of a box.  With C == 1 and W % 8 == 0 every 16-byte chunk is entirely inside
// or entirely outside the image (zeros).  Thread = (chunk c = tid & 31, row r = tid>>5 + 8k).
template <class Cfg>
__device__ __forceinline__ void stage_issue(const uint16_t* __restrict__ S, const Box& box, int H, int W, int tid,
                                            uint4 (&chunk)[Cfg::kRowPasses]) {
  const int cpr = box.pitch >> 3;
  const int sc = tid & 31, sr = tid >> 5;
  const int gx = box.ax0 + 8 * sc;
  const bool col_ok = sc < cpr && gx >= 0 && gx < W;
#pragma unroll
  for (int k = 0; k < Cfg::kRowPasses; ++k) {
    const int r = sr + 8 * k;
    const int gy = box.sy0 + r;
    chunk[k] = make_uint4(0u, 0u, 0u, 0u);
    if (r < box.rows && col_ok && (unsigned)gy < (unsigned)H)
      chunk[k] = *reinterpret_cast<const uint4*>(S + (size_t)gy * W + gx);
  }
}

template <class Cfg>
__device__ __forceinline__ void stage_land(uint16_t* stile, const Box& box, int tid,
                                           const uint4 (&chunk)[Cfg::kRowPasses]) {
  const int cpr = box.pitch >> 3;
  const int sc = tid & 31, sr = tid >> 5;
#pragma unroll
  for (int k = 0; k < Cfg::kRowPasses; ++k) {
    const int r = sr + 8 * k;
    if (r < box.rows && sc < cpr) *reinterpret_cast<uint4*>(&stile[r * box.pitch + 8 * sc]) = chunk[k];
  }
}

// Staging of a C-channel box with 16-byte chunks of the interleaved rows (W % 8 == 0:
// ax0 and W are multiples of 8 pixels, so a chunk is entirely inside or outside the
// image row and zero-filling whole chunks is exactly BORDER_CONSTANT).  Chunk
// q = tid + kThreads * k of the box; every load of a thread is issued before any lands
// (a load-then-store loop waits for each load in turn: the 4K RGB warp took 14.6 ms per
// 625 frames that way, 11.8 ms with the loads in flight together).
template <class Cfg, int C>
struct VecC {
  static constexpr int kPasses = (Cfg::kLdsElems / 8 + kThreads - 1) / kThreads;
};

template <class Cfg, int C>
__device__ __forceinline__ void stage_vec_c_issue(const uint16_t* __restrict__ S, const Box& box, int H, int W,
                                                  int tid, uint4 (&chunk)[VecC<Cfg, C>::kPasses]) {
  const int cpr = box.pitch * C / 8;
  const int total = box.rows * cpr;
  const int rowe = W * C;
#pragma unroll
  for (int k = 0; k < VecC<Cfg, C>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    const int r = q / cpr, cc = q - r * cpr;
    const int gy = box.sy0 + r;
    const int e = box.ax0 * C + 8 * cc;
    chunk[k] = make_uint4(0u, 0u, 0u, 0u);
    if (q < total && (unsigned)gy < (unsigned)H && e >= 0 && e < rowe)
      chunk[k] = *reinterpret_cast<const uint4*>(S + (size_t)gy * rowe + e);
  }
}

template <class Cfg, int C>
__device__ __forceinline__ void stage_vec_c_land(uint16_t* stile, const Box& box, int tid,
                                                 const uint4 (&chunk)[VecC<Cfg, C>::kPasses]) {
  const int total = box.rows * (box.pitch * C / 8);
#pragma unroll
  for (int k = 0; k < VecC<Cfg, C>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    if (q < total) reinterpret_cast<uint4*>(stile)[q] = chunk[k];
  }
}

// Element-wise staging (W % 8 != 0).
template <int C>
__device__ __forceinline__ void stage_scalar(const uint16_t* __restrict__ S, uint16_t* stile, const Box& box, int H,
                                             int W, int tid) {
  for (int q = tid; q < box.rows * box.pitch * C; q += kThreads) {
    const int r = q / (box.pitch * C), e = q - r * box.pitch * C;
    const int gy = box.sy0 + r, gx = box.ax0 + e / C, k = e % C;
    stile[q] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) ? S[((size_t)gy * W + gx) * C + k]
                                                                          : (uint16_t)0;
  }
}

// rint(S / 1024) (round half to even) for an integer S < 2^24, as the low 16 bits of
// fl(S * 2^-10 + 1.5 * 2^23): float(S) and the scaling are exact, the fused add rounds
// once to an integer (ulp 1 at that magnitude) in round-to-nearest-even.
__device__ __forceinline__ uint16_t round_q10(uint32_t S) {
  return (uint16_t)__float_as_uint(__builtin_fmaf((float)S, 0x1p-10f, 12582912.0f));
}

__device__ __forceinline__ uint32_t tap(const uint16_t* stile, int i) { return stile[i]; }

// Bits 11-15 of v in one v_bfe_u32 (a shift and a mask otherwise).  The builtin, not inline
// asm: the compiler pads the wait state a VALU write of a VGPR needs after a wider-than-8-byte
// store that reads it as data, but not around inline asm -- the round-4 inline-asm form landed
// right behind the RGB path's buffer_store_dwordx3 and overwrote its first data VGPR, an
// intermittent wrong pixel pair (tools/debug/store_hazard_scan.py checks the
// built library for that pattern).
__device__ __forceinline__ uint32_t bfe_11_5(uint32_t v) { return __builtin_amdgcn_ubfe(v, 11, 5); }


// Fast-path staging: chunk q = tid + 256k of the box in row-major order at kFastChunks
// chunks per row (LDS offset 16q); chunks right of the box's own pitch are left unwritten
// (never read).
template <class Cfg>
__device__ __forceinline__ void fast_stage_issue(const uint16_t* __restrict__ S, int ax0, int sy0, int cpr, int rows,
                                                 int H, int W, int tid, uint4 (&chunk)[Fast<Cfg>::kPasses]) {
#pragma unroll
  for (int k = 0; k < Fast<Cfg>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    const int r = q / kFastChunks, c = q - r * kFastChunks;
    const int gy = sy0 + r, gx = ax0 + 8 * c;
    chunk[k] = make_uint4(0u, 0u, 0u, 0u);
    if (r < rows && c < cpr && (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H)
      chunk[k] = *reinterpret_cast<const uint4*>(S + (size_t)gy * W + gx);
  }
}

template <class Cfg>
__device__ __forceinline__ void fast_stage_land(uint16_t* stile, int cpr, int rows, int tid,
                                                const uint4 (&chunk)[Fast<Cfg>::kPasses]) {
#pragma unroll
  for (int k = 0; k < Fast<Cfg>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    const int r = q / kFastChunks, c = q - r * kFastChunks;
    if (r < rows && c < cpr) reinterpret_cast<uint4*>(stile)[q] = chunk[k];
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// OpenCV's float evaluation of remapBilinear's blend, ((v00 w0 + v01 w1) + v10 w2) + v11 w3
// with separately rounded products and w_k = K_k / 1024 exactly (the 2^-10 scaling commutes
// with every rounding), then cvRound: packed fp32 over the lane's two pixels; returns the
// two results in the low 16 bits of each float.
__device__ __forceinline__ f32x2 blend_float2(const uint32_t (&v)[2][4], const uint32_t (&fx)[2],
                                              const uint32_t (&fy)[2]) {
  const f32x2 fxf = {(float)fx[0], (float)fx[1]}, fyf = {(float)fy[0], (float)fy[1]};
  const f32x2 axf = 32.0f - fxf, ayf = 32.0f - fyf;
  const f32x2 t0 = {(float)v[0][0], (float)v[1][0]}, t1 = {(float)v[0][1], (float)v[1][1]};
  const f32x2 t2 = {(float)v[0][2], (float)v[1][2]}, t3 = {(float)v[0][3], (float)v[1][3]};
  const f32x2 sum = ((t0 * (ayf * axf) + t1 * (ayf * fxf)) + t2 * (fyf * axf)) + t3 * (fyf * fxf);
  // cvRound(sum / 1024): one rounding of the exact sum * 2^-10 + 1.5 * 2^23
  f32x2 q;
  q[0] = __builtin_fmaf(sum[0], 0x1p-10f, 0x1.8p23f);
  q[1] = __builtin_fmaf(sum[1], 0x1p-10f, 0x1.8p23f);
  return q;
}

// Blend of a mode-3 tile, chosen once per tile from its staged box:
enum FastBlend {
  kDark = 0,    // every staged value < 16384: S = sum v_k K_k < 2^24, so the exact separable
                // integer evaluation of output_rows IS OpenCV's float result; no range check
  kMixed = 1,   // some bright values: per output row (wave-uniform), the integer blend when
                // all the row's taps are < 16384, blend_float2 otherwise
  kBright = 2,  // bright regions over much of the box: blend_float2 throughout
};
// kBright above this fraction of bright staged chunks: a float row costs ~1.25x an integer
// row, and a kMixed row pays ~10 % for its tap test (tools/warp_lab at config 2: dark
// 2.85 ms, all-bright 3.56 ms).
constexpr int kBrightShare = 3;  // bright chunks * kBrightShare > box chunks -> kBright

// Output rows of a mode-3 tile, with the per-row overheads of output_rows removed: row
// origins are scalar, the lower tap row is an immediate LDS offset, the store is a buffer
// store with the row offset in soffset.
// INTERIOR: the tile lies inside the frame (every row exists, every lane's pixel pair is
// stored), so the rows carry no bounds test and no store mask.
template <class Cfg, int BLEND, bool INTERIOR>
__device__ __forceinline__ void fast_rows(const uint16_t* stile, const int2* __restrict__ rt, int ox, int oy,
                                          uint16_t* __restrict__ Dst, int H, int W, int xb, int yb, int wave, int lane,
                                          const int (&ad)[2], const int (&bd)[2]) {
  const uint32_t xoff = 2u * (uint32_t)(xb + 2 * lane);  // byte offset of the lane's pixel pair
  const bool store_ok = INTERIOR || xb + 2 * lane + 2 <= W;  // W is even here
  const __amdgpu_buffer_rsrc_t dst_rsrc = __builtin_amdgcn_make_buffer_rsrc(Dst, 0, 2 * H * W, 0x00020000);
  int2 org[Cfg::kTileH / 4];  // all row origins up front (scalar loads; the table is padded)
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) org[i] = rt[i];
  // Box-relative coordinates are carried scaled by 2^6: the tap's integer column / row
  // (< 2^8 / 2^7 here) is then the high half of the word and the 1/32 fraction bits 11-15.
  // One v_perm packs (column, row) as two u16 and one v_dot2_u32_u16 with (2, 2 * pitch)
  // gives the tap's LDS byte offset (4 VALU per pixel fewer than shifts + mad).
  // Exact: |X| < 2^18 before scaling, and two's-complement wrap-around commutes with << 6.
  uint32_t ad6[2], bd6[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    ad6[p] = (uint32_t)ad[p] << 6;
    bd6[p] = (uint32_t)bd[p] << 6;
  }
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 pitch2 = {(unsigned short)2, (unsigned short)(2 * kFastPitch)};
  const char* sbytes = reinterpret_cast<const char*>(stile);
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) {
    const int y = yb + wave + 4 * i;  // wave-uniform
    if (!INTERIOR && y >= H) break;
    const uint32_t X0 = (uint32_t)(org[i].x - ox) << 6, Y0 = (uint32_t)(org[i].y - oy) << 6;  // scalar
    uint32_t v[2][4], fx[2], fy[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t tX = X0 + ad6[p], tY = Y0 + bd6[p];
      fx[p] = bfe_11_5(tX);
      fy[p] = bfe_11_5(tY);
      const uint32_t cr = __builtin_amdgcn_perm(tY, tX, 0x07060302u);  // (column, row) as u16 x 2
      const uint32_t off = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, cr), pitch2, 0u, false);
      const uint16_t* t = reinterpret_cast<const uint16_t*>(sbytes + off);
      v[p][0] = t[0];
      v[p][1] = t[1];
      v[p][2] = t[kFastPitch];
      v[p][3] = t[kFastPitch + 1];
    }
    bool use_float = BLEND == kBright;
    if constexpr (BLEND == kMixed) {
      const uint32_t taps = (v[0][0] | v[0][1] | v[0][2]) | (v[0][3] | v[1][0] | v[1][1]) | (v[1][2] | v[1][3]);
      use_float = __builtin_amdgcn_ballot_w64((taps & 0xc000u) != 0) != 0;  // wave-uniform
    }
    f32x2 q;
    if (use_float) {
      q = blend_float2(v, fx, fy);
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const uint32_t ax = 32 - fx[p], ay = 32 - fy[p];
        uint32_t h0 = __umul24(v[p][0], ax) + __umul24(v[p][1], fx[p]);
        uint32_t h1 = __umul24(v[p][2], ax) + __umul24(v[p][3], fx[p]);
        asm volatile("" : "+v"(h0), "+v"(h1));  // keep the separable form (see output_rows)
        q[p] = (float)(__umul24(h0, ay) + __umul24(h1, fy[p]));
      }
      // rint(S / 1024) in the low bits: fl(S) + 1.5 * 2^33 rounds (half to even) to a
      // multiple of 1024, the float's unit in the last place there
      q += 0x1.8p33f;
    }
    const uint32_t out = __builtin_amdgcn_perm(__float_as_uint(q[1]), __float_as_uint(q[0]), 0x05040100u);
    // aux 2 = nontemporal: the aligned frame is written once and not re-read here
    if (store_ok) __builtin_amdgcn_raw_buffer_store_b32(out, dst_rsrc, xoff, 2 * y * W, 2);
  }
}

// Fast staged path for C = 3 / 4 (mode 3 of a multi-channel frame, round 4).  The
// interleaved box is de-interleaved while it lands: each thread loads one 8-pixel group of
// a box row (C 16-byte chunks, 16-byte aligned because ax0 and W are multiples of 8) and
// writes C planar 16-byte pieces (v_perm_b32 pairs), one per channel plane, at the fixed
// pitch.  A pixel's taps then sit at the same offset in every plane (immediate offsets), so
// the coordinate work of a pixel is shared by its C channels, and each lane's C output
// dwords (pixels 2l, 2l+1) leave in ONE 12- / 16-byte store: a wave's store covers 768 /
// 1024 contiguous bytes of the row.  The general multi-channel path (mode 0) reads
// interleaved taps with per-channel addressing and stores C separate dwords per lane at a
// 12-byte lane stride (round 3: 148 VALU, 49 SALU, 25 LDS instructions per wave row at c4).
template <class Cfg, int C>
struct FastC {
  static constexpr int kPitch = 144;  // plane row pitch in pixels (192: fewer bank conflicts, same time)
  static constexpr int kRows = (Cfg::kLdsElems - 8) / (C * kPitch);      // the last 16 bytes: flags
  static constexpr int kPlane = kRows * kPitch;                          // elements per channel plane
  static constexpr int kFlagWord = Cfg::kLdsElems / 2 - 4;
  static constexpr int kGroups = kPitch / 8;                             // 8-pixel groups per staged row
  static constexpr int kPasses = (kRows * kGroups + kThreads - 1) / kThreads;
  static_assert(C * kPlane <= 2 * kFlagWord, "planes overlap the flag words");
};

template <class Cfg, int C>
__device__ __forceinline__ void fastc_stage_issue(const uint16_t* __restrict__ S, int ax0, int sy0, int gpr, int rows,
                                                  int H, int W, int tid,
                                                  uint4 (&g)[FastC<Cfg, C>::kPasses][C]) {
#pragma unroll
  for (int k = 0; k < FastC<Cfg, C>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    const int r = q / FastC<Cfg, C>::kGroups, c = q - r * FastC<Cfg, C>::kGroups;
    const int gy = sy0 + r, gx = ax0 + 8 * c;
    const bool ok = r < rows && c < gpr && (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
#pragma unroll
    for (int j = 0; j < C; ++j) g[k][j] = make_uint4(0u, 0u, 0u, 0u);
    if (ok) {
      const uint4* src = reinterpret_cast<const uint4*>(S + ((size_t)gy * W + gx) * C);
#pragma unroll
      for (int j = 0; j < C; ++j) g[k][j] = src[j];
    }
  }
}

// word i of plane k of an 8-pixel group: elements C (2i) + k and C (2i + 1) + k of the
// interleaved group (dwords d[e / 2], halves e % 2), as one v_perm_b32
template <int C, int K, int I>
__device__ __forceinline__ uint32_t plane_word(const uint32_t (&d)[4 * C]) {
  constexpr int e0 = C * 2 * I + K, e1 = C * (2 * I + 1) + K;
  constexpr uint32_t sel = ((e0 & 1) ? 0x0302u : 0x0100u) | ((e1 & 1) ? 0x07060000u : 0x05040000u);
  return __builtin_amdgcn_perm(d[e1 / 2], d[e0 / 2], sel);
}

template <int C, int K>
__device__ __forceinline__ uint4 plane_piece(const uint32_t (&d)[4 * C]) {
  return make_uint4(plane_word<C, K, 0>(d), plane_word<C, K, 1>(d), plane_word<C, K, 2>(d), plane_word<C, K, 3>(d));
}

template <class Cfg, int C>
__device__ __forceinline__ uint32_t fastc_stage_land(uint16_t* stile, int gpr, int rows, int tid,
                                                     const uint4 (&g)[FastC<Cfg, C>::kPasses][C]) {
  uint32_t nb = 0;  // bright (>= 16384) groups of this wave
#pragma unroll
  for (int k = 0; k < FastC<Cfg, C>::kPasses; ++k) {
    const int q = tid + kThreads * k;
    const int r = q / FastC<Cfg, C>::kGroups, c = q - r * FastC<Cfg, C>::kGroups;
    uint32_t d[4 * C], any = 0;  // the group's 8 C elements, two per dword
#pragma unroll
    for (int j = 0; j < C; ++j) {
      d[4 * j] = g[k][j].x;
      d[4 * j + 1] = g[k][j].y;
      d[4 * j + 2] = g[k][j].z;
      d[4 * j + 3] = g[k][j].w;
      any |= g[k][j].x | g[k][j].y | g[k][j].z | g[k][j].w;
    }
    nb += __builtin_popcountll(__builtin_amdgcn_ballot_w64((any & 0xc000c000u) != 0));
    if (r < rows && c < gpr) {
      uint4* dst = reinterpret_cast<uint4*>(stile + r * FastC<Cfg, C>::kPitch + 8 * c);
      dst[0] = plane_piece<C, 0>(d);
      dst[FastC<Cfg, C>::kPlane / 8] = plane_piece<C, 1>(d);
      dst[2 * FastC<Cfg, C>::kPlane / 8] = plane_piece<C, 2>(d);
      if constexpr (C == 4) dst[3 * FastC<Cfg, C>::kPlane / 8] = plane_piece<C, 3>(d);
    }
  }
  return nb;
}

// Output rows of a multi-channel mode-3 tile: fast_rows with C planes (same coordinate
// scheme, same three blends, the blend decided once per tile or per row over every
// channel's taps) and one b96 / b128 buffer store per lane and row.
template <class Cfg, int C, int BLEND, bool INTERIOR>
__device__ __forceinline__ void fastc_rows(const uint16_t* stile, const int2* __restrict__ rt, int ox, int oy,
                                           uint16_t* __restrict__ Dst, int H, int W, int xb, int yb, int wave,
                                           int lane, const int (&ad)[2], const int (&bd)[2]) {
  static_assert(C == 3 || C == 4, "planar fast path: RGB / RGBA");
  constexpr int kPlane = FastC<Cfg, C>::kPlane, kPitch = FastC<Cfg, C>::kPitch;
  const uint32_t xoff = 2u * C * (uint32_t)(xb + 2 * lane);  // byte offset of the lane's pixel pair
  const bool store_ok = INTERIOR || xb + 2 * lane + 2 <= W;   // W is a multiple of 8 here
  const __amdgpu_buffer_rsrc_t dst_rsrc = __builtin_amdgcn_make_buffer_rsrc(Dst, 0, 2 * C * H * W, 0x00020000);
  int2 org[Cfg::kTileH / 4];
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) org[i] = rt[i];
  uint32_t ad6[2], bd6[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    ad6[p] = (uint32_t)ad[p] << 6;
    bd6[p] = (uint32_t)bd[p] << 6;
  }
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 pitch2 = {(unsigned short)2, (unsigned short)(2 * kPitch)};
  const char* sbytes = reinterpret_cast<const char*>(stile);
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) {
    const int y = yb + wave + 4 * i;  // wave-uniform
    if (!INTERIOR && y >= H) break;
    const uint32_t X0 = (uint32_t)(org[i].x - ox) << 6, Y0 = (uint32_t)(org[i].y - oy) << 6;  // scalar
    uint32_t v[C][2][4], fx[2], fy[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t tX = X0 + ad6[p], tY = Y0 + bd6[p];
      fx[p] = bfe_11_5(tX);
      fy[p] = bfe_11_5(tY);
      const uint32_t cr = __builtin_amdgcn_perm(tY, tX, 0x07060302u);  // (column, row) as u16 x 2
      const uint32_t off = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, cr), pitch2, 0u, false);
      const uint16_t* t = reinterpret_cast<const uint16_t*>(sbytes + off);
#pragma unroll
      for (int k = 0; k < C; ++k) {
        v[k][p][0] = t[k * kPlane];
        v[k][p][1] = t[k * kPlane + 1];
        v[k][p][2] = t[k * kPlane + kPitch];
        v[k][p][3] = t[k * kPlane + kPitch + 1];
      }
    }
    bool use_float = BLEND == kBright;
    if constexpr (BLEND == kMixed) {
      uint32_t taps = 0;
#pragma unroll
      for (int k = 0; k < C; ++k)
        taps |= (v[k][0][0] | v[k][0][1] | v[k][0][2]) | (v[k][0][3] | v[k][1][0] | v[k][1][1]) |
                (v[k][1][2] | v[k][1][3]);
      use_float = __builtin_amdgcn_ballot_w64((taps & 0xc000u) != 0) != 0;  // wave-uniform
    }
    f32x2 q[C];
    if (use_float) {
#pragma unroll
      for (int k = 0; k < C; ++k) q[k] = blend_float2(v[k], fx, fy);
    } else {
#pragma unroll
      for (int k = 0; k < C; ++k) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint32_t ax = 32 - fx[p], ay = 32 - fy[p];
          uint32_t h0 = __umul24(v[k][p][0], ax) + __umul24(v[k][p][1], fx[p]);
          uint32_t h1 = __umul24(v[k][p][2], ax) + __umul24(v[k][p][3], fx[p]);
          asm volatile("" : "+v"(h0), "+v"(h1));  // keep the separable form (see output_rows)
          q[k][p] = (float)(__umul24(h0, ay) + __umul24(h1, fy[p]));
        }
        q[k] += 0x1.8p33f;  // rint(S / 1024) in the low bits (fast_rows)
      }
    }
    // the lane's 2 C channel values in interleaved order, two per dword
#define KCMC_Q(px, ch) __float_as_uint(q[ch][px])
    if constexpr (C == 3) {
      typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
      const u32x3 o = {__builtin_amdgcn_perm(KCMC_Q(0, 1), KCMC_Q(0, 0), 0x05040100u),
                       __builtin_amdgcn_perm(KCMC_Q(1, 0), KCMC_Q(0, 2), 0x05040100u),
                       __builtin_amdgcn_perm(KCMC_Q(1, 2), KCMC_Q(1, 1), 0x05040100u)};
      if (store_ok) __builtin_amdgcn_raw_buffer_store_b96(o, dst_rsrc, xoff, 2 * C * y * W, 2);
    } else {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 o = {__builtin_amdgcn_perm(KCMC_Q(0, 1), KCMC_Q(0, 0), 0x05040100u),
                       __builtin_amdgcn_perm(KCMC_Q(0, 3), KCMC_Q(0, 2), 0x05040100u),
                       __builtin_amdgcn_perm(KCMC_Q(1, 1), KCMC_Q(1, 0), 0x05040100u),
                       __builtin_amdgcn_perm(KCMC_Q(1, 3), KCMC_Q(1, 2), 0x05040100u)};
      if (store_ok) __builtin_amdgcn_raw_buffer_store_b128(o, dst_rsrc, xoff, 2 * C * y * W, 2);
    }
#undef KCMC_Q
  }
}

// Debug instrument (tools/debug/warp_sentinel.sh builds it; never the product library): the
// whole LDS array is filled with 0xFFFF before a tile stages its box, so that a tap read
// outside the staged rows / columns returns a deterministic wrong value (65535) instead of
// whatever an earlier workgroup left in that LDS, and the bit-exact tests catch it.
#ifdef KCMC_WARP_SENTINEL
template <int ELEMS>
__device__ __forceinline__ void lds_sentinel(uint16_t* stile, int tid) {
  for (int i = tid; i < ELEMS / 2; i += kThreads) reinterpret_cast<uint32_t*>(stile)[i] = 0xffffffffu;
  __syncthreads();
}
#define KCMC_LDS_SENTINEL(stile, elems, tid) lds_sentinel<elems>(stile, tid)
#else
#define KCMC_LDS_SENTINEL(stile, elems, tid) ((void)0)
#endif

// Per-tile plan made by warp_plan_kernel.
struct TilePlan {
  int mode, ax0, sy0;
  int pitch_rows;  // pitch | rows << 16
};

__device__ __forceinline__ Box unpack(const TilePlan& t) {
  Box b;
  b.mode = t.mode;
  b.ax0 = t.ax0;
  b.sy0 = t.sy0;
  b.pitch = t.pitch_rows & 0xffff;
  b.rows = t.pitch_rows >> 16;
  return b;
}

// Per-thread coordinates of one tile (WarpAffineInvoker): adelta/bdelta of the lane's two
// columns, and in lane i < kTileH/4 the row origins X0/Y0 of the wave's i-th row.  For a
// staged tile the box origin (ox, oy) is folded into the row origins (a multiple of 1024
// in fixed point, so the fractional bits are unchanged): coordinates are box-relative.
// Columns past the frame edge reuse the last valid column's coordinates so that their
// (never stored) taps stay inside the box.
__device__ __forceinline__ void lane_cols(const double* __restrict__ M, int xb, int W, int lane, int (&ad)[2],
                                          int (&bd)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int x = min(xb + 2 * lane + q, W - 1);
    ad[q] = cv_round(M[0] * x * 1024);
    bd[q] = cv_round(M[3] * x * 1024);
  }
}

template <class Cfg>
__device__ __forceinline__ void lane_coords(const double* __restrict__ M, int xb, int yb, int W, int wave, int lane,
                                            int ox, int oy, int (&ad)[2], int (&bd)[2], int& X0v, int& Y0v) {
  lane_cols(M, xb, W, lane, ad, bd);
  const int y = yb + wave + 4 * min(lane, Cfg::kTileH / 4 - 1);
  X0v = cv_round((M[1] * y + M[2]) * 1024) + 16 - ox * 1024;
  Y0v = cv_round((M[4] * y + M[5]) * 1024) + 16 - oy * 1024;
}

// Output rows of one tile on one path (0: LDS-staged box, 1: zeros, 2: direct gather).
// Wave w makes rows w, w + 4, ...; lane l pixels x = xb + 2l, xb + 2l + 1.
template <class Cfg, int C, int MODE>
__device__ __forceinline__ void output_rows(const uint16_t* stile, const Box& box, const uint16_t* __restrict__ S,
                                            uint16_t* __restrict__ Dst, int H, int W, int xb, int yb, int wave,
                                            int lane, const int (&ad)[2], const int (&bd)[2], int X0v, int Y0v) {
  const int x = xb + 2 * lane;
  const bool pair_store = C == 1 && (W & 1) == 0 && x + 2 <= W;
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) {
    const int y = yb + wave + 4 * i;  // wave-uniform
    if (y >= H) break;
    const int X0 = __builtin_amdgcn_readlane(X0v, i), Y0 = __builtin_amdgcn_readlane(Y0v, i);
    uint16_t o[2 * C];
    if (MODE == 0) {
      // Box-relative taps.  The blend is first evaluated exactly in integers,
      // S = ay*(v00*ax + v01*fx) + fy*(v10*ax + v11*fx) = sum v_k*K_k: while S < 2^24
      // every product and partial sum of OpenCV's float evaluation is an integer below
      // 2^24 as well, hence exact, and its result is rint(S/1024).  Only pixels with
      // S >= 2^24 (bright: taps beyond 14 bits) take the float-faithful blend.
      uint32_t Sx[2 * C], hi = 0, fx[2], fy[2], li[2], v[2][C][4];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int tX = X0 + ad[p], tY = Y0 + bd[p];
        fx[p] = (tX >> 5) & 31;
        fy[p] = (tY >> 5) & 31;
        li[p] = __umul24((uint32_t)(tY >> 10), (uint32_t)box.pitch) + (uint32_t)(tX >> 10);
      }
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < C; ++k) {
          const int i00 = li[p] * C + k, i10 = i00 + box.pitch * C;
          v[p][k][0] = tap(stile, i00);
          v[p][k][1] = tap(stile, i00 + C);
          v[p][k][2] = tap(stile, i10);
          v[p][k][3] = tap(stile, i10 + C);
        }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const uint32_t ax = 32 - fx[p], ay = 32 - fy[p];
#pragma unroll
        for (int k = 0; k < C; ++k) {
          uint32_t h0 = __umul24(v[p][k][0], ax) + __umul24(v[p][k][1], fx[p]);
          uint32_t h1 = __umul24(v[p][k][2], ax) + __umul24(v[p][k][3], fx[p]);
          // keep the separable form (the compiler would otherwise expand it into the
          // four weight products, three more multiplies)
          asm volatile("" : "+v"(h0), "+v"(h1));
          const uint32_t Sv = __umul24(h0, ay) + __umul24(h1, fy[p]);
          Sx[p * C + k] = Sv;
          hi |= Sv;
          o[p * C + k] = round_q10(Sv);
        }
      }
      if (hi >> 24) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int k = 0; k < C; ++k)
            if (Sx[p * C + k] >> 24)
              o[p * C + k] = blend_int(v[p][k][0], v[p][k][1], v[p][k][2], v[p][k][3], fx[p], fy[p]);
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int X = (X0 + ad[p]) >> 5, Y = (Y0 + bd[p]) >> 5;
        if (MODE == 1) {
#pragma unroll
          for (int k = 0; k < C; ++k) o[p * C + k] = 0;
        } else {
          bilinear_px<C>(S, H, W, X, Y, o + p * C);
        }
      }
    }
    uint16_t* drow = Dst + ((size_t)y * W + x) * C;
    if (pair_store) {
      // streaming store: the aligned frame is written once and not re-read by this kernel
      __builtin_nontemporal_store((uint32_t)o[0] | ((uint32_t)o[1] << 16), reinterpret_cast<uint32_t*>(drow));
    } else if (C >= 3 && x + 2 <= W) {
      // two whole pixels: 6 (RGB) or 8 (RGBA) channels as 4-byte stores (x even -> aligned)
#pragma unroll
      for (int k = 0; k < C; ++k)
        __builtin_nontemporal_store((uint32_t)o[2 * k] | ((uint32_t)o[2 * k + 1] << 16),
                                    reinterpret_cast<uint32_t*>(drow) + k);
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (x + q < W)
#pragma unroll
          for (int k = 0; k < C; ++k) drow[q * C + k] = o[q * C + k];
    }
  }
}

// One row loop per path (a path-uniform branch inside the loop makes the compiler drain
// the previous rows' stores with s_waitcnt vmcnt(0) every row).
template <class Cfg, int C>
__device__ __forceinline__ void output_tile(int mode, const uint16_t* stile, const Box& box,
                                            const uint16_t* __restrict__ S, uint16_t* __restrict__ Dst, int H, int W,
                                            int xb, int yb, int wave, int lane, const int (&ad)[2], const int (&bd)[2],
                                            int X0v, int Y0v) {
  if (mode == 0)
    output_rows<Cfg, C, 0>(stile, box, S, Dst, H, W, xb, yb, wave, lane, ad, bd, X0v, Y0v);
  else if (mode == 1)
    output_rows<Cfg, C, 1>(stile, box, S, Dst, H, W, xb, yb, wave, lane, ad, bd, X0v, Y0v);
  else
    output_rows<Cfg, C, 2>(stile, box, S, Dst, H, W, xb, yb, wave, lane, ad, bd, X0v, Y0v);
}

// (xcd_remap: kcmc_internal.h)

// ------------------------------------------------------------------------- plan
// One thread per tile (tile id = (f * nty + ty) * ntx + tx): the fp64 map inversion
// (written once per frame to minv) and the tile's source box.
// Also the frame's row-origin table for the fast path: rowtab[f][y & 3][y >> 2] =
// (X0(y), Y0(y)) = (cvRound((M1*y + M2)*1024) + 16, cvRound((M4*y + M5)*1024) + 16), so
// that a wave's rows y = yb + wave + 4i are consecutive entries; the tiles of a tile row
// share its rows.
template <int C, class Cfg>
__global__ __launch_bounds__(256) void warp_plan_kernel(const double* __restrict__ Mall, int n_frames, int H, int W,
                                                        int inverse_map, int ntx, int nty,
                                                        TilePlan* __restrict__ plan, double* __restrict__ minv,
                                                        int2* __restrict__ rowtab, int hq) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)ntx * nty * n_frames) return;
  const int f = (int)(t / (ntx * nty)), t2 = (int)(t - (long long)f * ntx * nty);
  const int tx = t2 % ntx, xb = tx * kTileW, yb = (t2 / ntx) * Cfg::kTileH;
  double M[6];
  load_map(Mall, f, inverse_map, M);
  if (t2 == 0)
    for (int k = 0; k < 6; ++k) minv[6 * (size_t)f + k] = M[k];
  Box b = source_box<Cfg, C>(M, xb, yb, H, W);
  if constexpr (C == 1) {
    if ((W & 7) == 0 && b.mode == 0 && b.pitch <= kFastPitch && b.rows <= Fast<Cfg>::kRows) b.mode = 3;
  } else if constexpr (C == 3 || C == 4) {
    if ((W & 7) == 0 && b.mode == 0 && b.pitch <= FastC<Cfg, C>::kPitch && b.rows <= FastC<Cfg, C>::kRows) b.mode = 3;
  }
  if (map_has_nan(M, 6)) b.mode = 1;  // a NaN map (a frame RANSAC could not fit) warps to zeros
  plan[t] = TilePlan{b.mode, b.ax0, b.sy0, b.pitch | (b.rows << 16)};
  for (int j = tx; j < Cfg::kTileH && yb + j < H; j += ntx) {
    const int y = yb + j;
    rowtab[((size_t)f * 4 + (y & 3)) * hq + (y >> 2)] =
        make_int2(cv_round((M[1] * y + M[2]) * 1024) + 16, cv_round((M[4] * y + M[5]) * 1024) + 16);
  }
}

// ------------------------------------------------------------ one tile per workgroup
// no-unaligned-access-mode: keeps the two adjacent 16-bit tap reads from being fused
// into one 4-byte LDS read at a 2-byte-aligned address, which the LDS replays (1.75x
// slower kernel, measured in tools/warp_lab).
template <int C, class Cfg = BlockCfg>
__global__ __launch_bounds__(kThreads) __attribute__((target("no-unaligned-access-mode"))) void warp_affine_u16_kernel(
    const uint16_t* __restrict__ src, uint16_t* __restrict__ dst, const TilePlan* __restrict__ plan,
    const double* __restrict__ minv, const int2* __restrict__ rowtab, int hq, int H, int W) {
  __shared__ __attribute__((aligned(16))) uint16_t stile[Cfg::kLdsElems];
  const int ntx = gridDim.x, nty = gridDim.y;
  const int tile = xcd_remap(blockIdx.x + ntx * (blockIdx.y + nty * blockIdx.z), ntx * nty * gridDim.z);
  const int f = tile / (ntx * nty);
  const int t2 = tile - f * ntx * nty;
  const int xb = (t2 % ntx) * kTileW, yb = (t2 / ntx) * Cfg::kTileH;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const uint16_t* S = src + (size_t)f * H * W * C;
  uint16_t* Dst = dst + (size_t)f * H * W * C;

  Box box = unpack(plan[tile]);
  KCMC_LDS_SENTINEL(stile, Cfg::kLdsElems, tid);
  if constexpr (C == 1) {
    if (box.mode == 3) {
      const int cpr = box.pitch >> 3;
      uint4 fchunk[Fast<Cfg>::kPasses];
      fast_stage_issue<Cfg>(S, box.ax0, box.sy0, cpr, box.rows, H, W, tid, fchunk);  // loads first
      int ad[2], bd[2];
      lane_cols(minv + 6 * (size_t)f, xb, W, lane, ad, bd);
      fast_stage_land<Cfg>(stile, cpr, box.rows, tid, fchunk);
      // bright (>= 16384) staged chunks of the box, counted per wave into the flag words
      uint32_t nb = 0;
#pragma unroll
      for (int k = 0; k < Fast<Cfg>::kPasses; ++k)
        nb += __builtin_popcountll(__builtin_amdgcn_ballot_w64(
            ((fchunk[k].x | fchunk[k].y | fchunk[k].z | fchunk[k].w) & 0xc000c000u) != 0));
      uint32_t* flags = reinterpret_cast<uint32_t*>(stile) + Fast<Cfg>::kFlagWord;
      if (lane == 0) flags[wave] = nb;
      __syncthreads();
      const uint4 fl = *reinterpret_cast<const uint4*>(flags);
      const uint32_t bright = fl.x + fl.y + fl.z + fl.w;
      const int2* rt = rowtab + ((size_t)f * 4 + wave) * hq + (yb >> 2);
      const int ox = box.ax0 * 1024, oy = box.sy0 * 1024;
      const bool interior = yb + Cfg::kTileH <= H && xb + kTileW <= W;
      if (bright == 0) {
        if (interior)
          fast_rows<Cfg, kDark, true>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
        else
          fast_rows<Cfg, kDark, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      } else if ((int)bright * kBrightShare <= box.rows * (box.pitch >> 3)) {
        if (interior)
          fast_rows<Cfg, kMixed, true>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
        else
          fast_rows<Cfg, kMixed, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      } else {
        fast_rows<Cfg, kBright, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      }
      return;
    }
  }
  if constexpr (C == 3 || C == 4) {
    if (box.mode == 3) {
      const int gpr = box.pitch >> 3;
      uint4 g[FastC<Cfg, C>::kPasses][C];
      fastc_stage_issue<Cfg, C>(S, box.ax0, box.sy0, gpr, box.rows, H, W, tid, g);  // loads first
      int ad[2], bd[2];
      lane_cols(minv + 6 * (size_t)f, xb, W, lane, ad, bd);
      const uint32_t nb = fastc_stage_land<Cfg, C>(stile, gpr, box.rows, tid, g);
      uint32_t* flags = reinterpret_cast<uint32_t*>(stile) + FastC<Cfg, C>::kFlagWord;
      if (lane == 0) flags[wave] = nb;
      __syncthreads();
      const uint4 fl = *reinterpret_cast<const uint4*>(flags);
      const uint32_t bright = fl.x + fl.y + fl.z + fl.w;
      const int2* rt = rowtab + ((size_t)f * 4 + wave) * hq + (yb >> 2);
      const int ox = box.ax0 * 1024, oy = box.sy0 * 1024;
      const bool interior = yb + Cfg::kTileH <= H && xb + kTileW <= W;
      if (bright == 0) {
        if (interior)
          fastc_rows<Cfg, C, kDark, true>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
        else
          fastc_rows<Cfg, C, kDark, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      } else if ((int)bright * kBrightShare <= box.rows * (box.pitch >> 3)) {
        if (interior)
          fastc_rows<Cfg, C, kMixed, true>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
        else
          fastc_rows<Cfg, C, kMixed, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      } else {
        fastc_rows<Cfg, C, kBright, false>(stile, rt, ox, oy, Dst, H, W, xb, yb, wave, lane, ad, bd);
      }
      return;
    }
  }
  const bool vec_stage = (C == 1) && ((W & 7) == 0);
  uint4 chunk[Cfg::kRowPasses];
  uint4 cchunk[C > 1 ? VecC<Cfg, C>::kPasses : 1];
  if (box.mode == 0 && vec_stage) stage_issue<Cfg>(S, box, H, W, tid, chunk);  // loads first
  if constexpr (C > 1) {
    if (box.mode == 0 && (W & 7) == 0) stage_vec_c_issue<Cfg, C>(S, box, H, W, tid, cchunk);
  }
  int ad[2], bd[2], X0v, Y0v;  // overlaps the loads
  lane_coords<Cfg>(minv + 6 * (size_t)f, xb, yb, W, wave, lane, box.mode == 0 ? box.ax0 : 0,
                   box.mode == 0 ? box.sy0 : 0, ad, bd, X0v, Y0v);
  if (box.mode == 0) {
    if (vec_stage) {
      stage_land<Cfg>(stile, box, tid, chunk);
    } else if (C > 1 && (W & 7) == 0) {
      if constexpr (C > 1) stage_vec_c_land<Cfg, C>(stile, box, tid, cchunk);
    } else {
      stage_scalar<C>(S, stile, box, H, W, tid);
    }
  }
  __syncthreads();
  output_tile<Cfg, C>(box.mode, stile, box, S, Dst, H, W, xb, yb, wave, lane, ad, bd, X0v, Y0v);
}

// Row-origin table entries per (frame, y & 3): padded so that a wave's scalar loads of
// its kTileH / 4 entries stay inside the frame's block.
inline int rowtab_hq(int H) { return ceil_div(H, 4) + 16; }

template <class Cfg>
size_t warp_workspace_bytes(int n_frames, int H, int W) {
  const size_t tiles = (size_t)ceil_div(W, kTileW) * ceil_div(H, Cfg::kTileH) * n_frames;
  return tiles * sizeof(TilePlan) + (size_t)n_frames * 6 * sizeof(double) +
         (size_t)n_frames * 4 * rowtab_hq(H) * sizeof(int2);
}

// Workspace layout of the affine warp: minv [F, 6] f64, rowtab [F, 4, hq] int2, plan [tiles].
template <class Cfg>
struct WarpWs {
  double* minv;
  int2* rowtab;
  TilePlan* plan;
  int hq;
  WarpWs(void* ws, int n_frames, int H) {
    minv = static_cast<double*>(ws);
    hq = rowtab_hq(H);
    rowtab = reinterpret_cast<int2*>(minv + 6 * (size_t)n_frames);
    plan = reinterpret_cast<TilePlan*>(rowtab + (size_t)n_frames * 4 * hq);
  }
};

template <int C, class Cfg = typename CfgFor<C>::type>
void launch_warp_plan(const double* M, int n_frames, int H, int W, int inverse_map, void* ws, hipStream_t s) {
  const int ntx = ceil_div(W, kTileW), nty = ceil_div(H, Cfg::kTileH);
  const long long tiles = (long long)ntx * nty * n_frames;
  const WarpWs<Cfg> w(ws, n_frames, H);
  hipLaunchKernelGGL((warp_plan_kernel<C, Cfg>), dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, s, M, n_frames,
                     H, W, inverse_map, ntx, nty, w.plan, w.minv, w.rowtab, w.hq);
}

template <int C, class Cfg = typename CfgFor<C>::type>
void launch_warp_tiles(const uint16_t* src, uint16_t* dst, int n_frames, int H, int W, const void* ws, hipStream_t s) {
  const int ntx = ceil_div(W, kTileW), nty = ceil_div(H, Cfg::kTileH);
  const WarpWs<Cfg> w(const_cast<void*>(ws), n_frames, H);
  hipLaunchKernelGGL((warp_affine_u16_kernel<C, Cfg>), dim3(ntx, nty, n_frames), dim3(kThreads), 0, s, src,
                     dst, w.plan, w.minv, w.rowtab, w.hq, H, W);
}

// Plan + tile launches on `s`; ws holds warp_workspace_bytes<Cfg>(n_frames, H, W) bytes.
template <int C, class Cfg = typename CfgFor<C>::type>
void launch_warp(const uint16_t* src, uint16_t* dst, const double* M, int n_frames, int H, int W, int inverse_map,
                 void* ws, hipStream_t s) {
  launch_warp_plan<C, Cfg>(M, n_frames, H, W, inverse_map, ws, s);
  launch_warp_tiles<C, Cfg>(src, dst, n_frames, H, W, ws, s);
}

// ================================================================ warpPerspective
// cv2.warpPerspective(frame, H, (W, H), INTER_LINEAR), BORDER_CONSTANT 0 -- the warp of
// the homography extension (BASELINE config 5; the reference only calls warpAffine).
// OpenCV classic path: invert(M) (closed-form 3x3, core/src/lapack.cpp) unless
// WARP_INVERSE_MAP, then WarpPerspectiveInvoker (imgwarp.cpp) per block of bw0 columns:
//   X0 = M0*xo + M1*y + M2, Y0 = M3*xo + M4*y + M5, W0 = M6*xo + M7*y + M8  (xo = block's
//   first column, x1 = x - xo), W = W0 + M6*x1, W = W ? 32/W : 0,
//   X = cvRound(clamp((X0 + M0*x1)*W)), Y likewise -> 1/32-px coordinates,
// and the same remapBilinear blend as warpAffine.  The coordinates are not separable,
// so each pixel evaluates them in fp64; the tile machinery (plan, LDS-staged box,
// exact integer blend, direct gather, zeros) is the affine kernel's.

__device__ __forceinline__ void invert_perspective(const double* S, double* M) {
  double d = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) +
             S[2] * (S[3] * S[7] - S[4] * S[6]);
  if (d == 0.0) {
    for (int k = 0; k < 9; ++k) M[k] = 0.0;
    return;
  }
  d = 1. / d;
  M[0] = (S[4] * S[8] - S[5] * S[7]) * d;
  M[1] = (S[2] * S[7] - S[1] * S[8]) * d;
  M[2] = (S[1] * S[5] - S[2] * S[4]) * d;
  M[3] = (S[5] * S[6] - S[3] * S[8]) * d;
  M[4] = (S[0] * S[8] - S[2] * S[6]) * d;
  M[5] = (S[2] * S[3] - S[0] * S[5]) * d;
  M[6] = (S[3] * S[7] - S[4] * S[6]) * d;
  M[7] = (S[1] * S[6] - S[0] * S[7]) * d;
  M[8] = (S[0] * S[4] - S[1] * S[3]) * d;
}

// Per-tile row table of the perspective warp (round 4): WarpPerspectiveInvoker's per-(row,
// block) values X0 = M0 xo + M1 y + M2, Y0 = M3 xo + M4 y + M5, W0 = M6 xo + M7 y + M8 for
// the tile's kTileH rows and its two 64-column blocks (bw0 = 64 for every frame with
// H >= 16 and W >= 64), computed once per workgroup into the last bytes of the LDS budget
// instead of by every lane for every row (9 of a row's 39 fp64 operations per lane); the
// staged box gets the budget minus the table.
template <class Cfg>
struct PerspTab {
  static constexpr int kEntries = Cfg::kTileH * 2;                  // (row, block)
  static constexpr int kElems = kEntries * 3 * 4;                   // u16 elements of 3 doubles each
  static constexpr int kFlagWord = Cfg::kLdsElems / 2 - 4;          // the last 16 bytes: per-wave flags
  static constexpr int kBoxElems = Cfg::kLdsElems - 8 - kElems;     // the staged box's budget
  static_assert((kBoxElems * 2) % 8 == 0, "table alignment");
};

// Source box of a tile: when the projective denominator has one sign over the tile,
// the tile's image is the convex hull of its corner images; one pixel of margin on each
// side absorbs the 1/32-px rounding and the second tap.  Otherwise: direct gather.
template <class Cfg, int C>
__device__ __forceinline__ Box persp_box(const double* M, int xb, int yb, int H, int W) {
  const int xl = min(xb + kTileW, W) - 1, yl = min(yb + Cfg::kTileH, H) - 1;
  const int cx[4] = {xb, xl, xb, xl}, cy[4] = {yb, yb, yl, yl};
  double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY;
  bool pos = true, neg = true, wrange = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double w = M[6] * cx[k] + M[7] * cy[k] + M[8];
    pos = pos && w > 0.0;
    neg = neg && w < 0.0;
    // the staged path's division assumes 2^-60 <= |w| <= 2^60 (w is linear over the tile:
    // its extremes are at the corners; a factor 2^4 of margin for the rounding)
    wrange = wrange && fabs(w) >= 0x1p-56 && fabs(w) <= 0x1p56;
    const double sx = (M[0] * cx[k] + M[1] * cy[k] + M[2]) / w;
    const double sy = (M[3] * cx[k] + M[4] * cy[k] + M[5]) / w;
    mnx = fmin(mnx, sx);
    mxx = fmax(mxx, sx);
    mny = fmin(mny, sy);
    mxy = fmax(mxy, sy);
  }
  Box b;
  b.mode = 2;
  b.ax0 = b.sy0 = b.pitch = b.rows = 0;
  const double lim = 30000.0;  // keep clear of saturate_cast<short> on coordinates
  if (!(pos || neg) || !(mnx > -lim && mxx < lim && mny > -lim && mxy < lim)) return b;
  const long long sx0 = (long long)floor(mnx) - 1, sx1 = (long long)floor(mxx) + 2;
  const long long sy0 = (long long)floor(mny) - 1, sy1 = (long long)floor(mxy) + 2;
  const long long ax0 = (sx0 >> 3) << 3;
  const long long pitch = ((sx1 - ax0 + 1) + 7) & ~7ll;
  const long long rows = sy1 - sy0 + 1;
  if (sx1 < 0 || sx0 > W - 1 || sy1 < 0 || sy0 > H - 1)
    b.mode = 1;
  else if (wrange && pitch <= kMaxPitch && rows <= 8 * Cfg::kRowPasses && pitch * rows * C <= PerspTab<Cfg>::kBoxElems)
    b.mode = 0;
  b.ax0 = (int)ax0;
  b.sy0 = (int)sy0;
  b.pitch = (int)pitch;
  b.rows = (int)rows;
  return b;
}

template <int C, class Cfg>
__global__ __launch_bounds__(256) void persp_plan_kernel(const double* __restrict__ Mall, int n_frames, int H, int W,
                                                         int inverse_map, int ntx, int nty, TilePlan* __restrict__ plan,
                                                         double* __restrict__ minv) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)ntx * nty * n_frames) return;
  const int f = (int)(t / (ntx * nty)), t2 = (int)(t - (long long)f * ntx * nty);
  const int xb = (t2 % ntx) * kTileW, yb = (t2 / ntx) * Cfg::kTileH;
  double M[9];
  if (inverse_map) {
    for (int k = 0; k < 9; ++k) M[k] = Mall[9 * (size_t)f + k];
  } else {
    invert_perspective(Mall + 9 * (size_t)f, M);
  }
  if (t2 == 0)
    for (int k = 0; k < 9; ++k) minv[9 * (size_t)f + k] = M[k];
  Box b = persp_box<Cfg, C>(M, xb, yb, H, W);
  if (map_has_nan(M, 9)) b.mode = 1;  // a NaN map (a frame RANSAC could not fit) warps to zeros
  plan[t] = TilePlan{b.mode, b.ax0, b.sy0, b.pitch | (b.rows << 16)};
}

// remapBilinear's blend of four taps: exact integer evaluation, with the float-faithful
// re-blend for sums >= 2^24 (see output_rows).
__device__ __forceinline__ uint16_t blend_exact(uint32_t v00, uint32_t v01, uint32_t v10, uint32_t v11, int fx,
                                                int fy) {
  const uint32_t ax = 32 - fx, ay = 32 - fy;
  uint32_t h0 = __umul24(v00, ax) + __umul24(v01, (uint32_t)fx);
  uint32_t h1 = __umul24(v10, ax) + __umul24(v11, (uint32_t)fx);
  asm volatile("" : "+v"(h0), "+v"(h1));
  const uint32_t Sv = __umul24(h0, ay) + __umul24(h1, (uint32_t)fy);
  uint16_t r = round_q10(Sv);
  if (Sv >> 24) r = blend_int(v00, v01, v10, v11, fx, fy);
  return r;
}

// WarpPerspectiveInvoker's fixed-point source coordinate of an output pixel from its
// per-(block, row) values X0, Y0, W0 (xo = the first column of the pixel's bw0-wide block)
// and the column's products M0 x1, M3 x1, M6 x1 (x1 = x - xo) -- the same values OpenCV
// computes, so the result is unchanged: W = W0 + M6 x1, W = W ? 32/W : 0,
// X = cvRound(clamp((X0 + M0 x1) W)), Y likewise.  IN_RANGE: the tile's plan has bounded
// every source coordinate of the tile within +-30000 px (a staged box), so OpenCV's clamp
// to [INT_MIN, INT_MAX] is the identity and is left out.
// 32 / w correctly rounded for 2^-60 <= |w| <= 2^60: the compiler's IEEE division sequence
// without its range scaling (v_div_scale leaves both operands unscaled in that range and
// v_div_fmas is then a plain fma) and without v_div_fixup (special values only): the same
// reciprocal, two Newton steps, quotient, residual and correction, so the same bits.
__device__ __forceinline__ double div32_in_range(double w) {
  double y = __builtin_amdgcn_rcp(w);
  double e = __builtin_fma(-w, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-w, y, 1.0);
  y = __builtin_fma(y, e, y);
  const double q = 32.0 * y;
  const double r = __builtin_fma(-w, q, 32.0);
  return __builtin_fma(r, y, q);
}

// rint(x) for |x| < 2^31 as the low word of x + 1.5 * 2^52 (one round-to-nearest-even add
// to an integer-ulp binade; two's complement for negative x)
__device__ __forceinline__ int rint_small(double x) {
  return (int)(uint32_t)__double_as_longlong(x + 0x1.8p52);
}

// The staged path's coordinates relative to the box origin (cx = 1.5 * 2^52 - 32 ax0,
// cy = 1.5 * 2^52 - 32 sy0): the low word of fl(fX) + cx is rint(fX) - 32 ax0, because the
// constant is an even integer in the binade of unit ulp (the add's tie-to-even is rint's).
__device__ __forceinline__ void persp_px_box(double X0, double Y0, double W0, double m0x1, double m3x1, double m6x1,
                                             double cx, double cy, uint32_t& X, uint32_t& Y) {
  const double w = div32_in_range(W0 + m6x1);
  X = (uint32_t)__double_as_longlong((X0 + m0x1) * w + cx);
  Y = (uint32_t)__double_as_longlong((Y0 + m3x1) * w + cy);
}

template <bool IN_RANGE>
__device__ __forceinline__ void persp_px(double X0, double Y0, double W0, double m0x1, double m3x1, double m6x1,
                                         int& X, int& Y) {
  double w = W0 + m6x1;
  if (IN_RANGE) {
    // staged tiles: the plan kept |w| within [2^-60, 2^60] and every coordinate within
    // +-30000 px, so the division needs no range handling and OpenCV's clamp to
    // [INT_MIN, INT_MAX] is the identity
    w = div32_in_range(w);
    X = rint_small((X0 + m0x1) * w);
    Y = rint_small((Y0 + m3x1) * w);
    return;
  }
  w = w != 0.0 ? 32.0 / w : 0.0;
  double fX = (X0 + m0x1) * w, fY = (Y0 + m3x1) * w;
  fX = fmax((double)INT_MIN, fmin((double)INT_MAX, fX));
  fY = fmax((double)INT_MIN, fmin((double)INT_MAX, fY));
  X = (int)__builtin_rint(fX);
  Y = (int)__builtin_rint(fY);
}

// DARK (MODE 0, C == 1): every staged value is < 16384, so the exact integer blend needs no
// range check (as kDark of the affine fast path).
template <class Cfg, int C, int MODE, bool TAB, bool DARK = false>
__device__ __forceinline__ void persp_rows(const uint16_t* stile, const Box& box, const uint16_t* __restrict__ S,
                                           uint16_t* __restrict__ Dst, const double* M, int H, int W, int xb, int yb,
                                           int wave, int lane, int bw0, const double* ptab) {
  const int x = xb + 2 * lane;
  const bool pair_store = C == 1 && (W & 1) == 0 && x + 2 <= W;
  int xo[2], x1[2], tb[2];
  double m0x1[2], m3x1[2], m6x1[2], dxo[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int xc = min(x + q, W - 1);  // columns past the edge reuse the last column's taps
    xo[q] = xc - xc % bw0;
    x1[q] = xc - xo[q];
    tb[q] = (xo[q] - xb) >> 6;  // TAB (bw0 == 64): the pixel's block of the tile (0 or 1)
    // row-invariant: the column products and the block origin (round 3: hoisted out of
    // the row loop, and X0 / Y0 / W0 evaluated once per row for the lane's pixel pair)
    m0x1[q] = M[0] * x1[q];
    m3x1[q] = M[3] * x1[q];
    m6x1[q] = M[6] * x1[q];
    dxo[q] = (double)xo[q];
  }
  const bool one_block = xo[0] == xo[1];  // the pair straddles a block edge only for odd bw0
  const double mx0 = M[0] * dxo[0], mx3 = M[3] * dxo[0], mx6 = M[6] * dxo[0];
  // MODE 0, C == 1: box-relative fixed-point taps; (column, row) packed as two u16 from the
  // coordinates shifted by 11 (bits 16+: the pixel, bits 11-15: the 1/32 fraction) and the
  // LDS byte offset as one v_dot2 with (2, 2 pitch) -- as fast_rows (the generic form costs a
  // quarter-rate v_mul_lo_u32 and two more subtractions per tap)
  const double cx = 0x1.8p52 - 32.0 * box.ax0, cy = 0x1.8p52 - 32.0 * box.sy0;
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 pitch2 = {(unsigned short)2, (unsigned short)(2 * box.pitch)};
  const char* sbytes = reinterpret_cast<const char*>(stile);
#pragma unroll
  for (int i = 0; i < Cfg::kTileH / 4; ++i) {
    const int y = yb + wave + 4 * i;  // wave-uniform
    if (y >= H) break;
    uint16_t o[2 * C];
    const double dy = (double)y;
    double X0[2], Y0[2], W0[2];
    if (TAB) {  // the workgroup's table (same expressions, evaluated once per (row, block))
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const double* e = ptab + 3 * (2 * (wave + 4 * i) + tb[p]);
        X0[p] = e[0];
        Y0[p] = e[1];
        W0[p] = e[2];
      }
    } else {
      X0[0] = mx0 + M[1] * dy + M[2];
      Y0[0] = mx3 + M[4] * dy + M[5];
      W0[0] = mx6 + M[7] * dy + M[8];
      X0[1] = X0[0];
      Y0[1] = Y0[0];
      W0[1] = W0[0];
      if (!one_block) {
        X0[1] = M[0] * dxo[1] + M[1] * dy + M[2];
        Y0[1] = M[3] * dxo[1] + M[4] * dy + M[5];
        W0[1] = M[6] * dxo[1] + M[7] * dy + M[8];
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if constexpr (MODE == 0 && C == 1) {
        uint32_t X, Y;
        persp_px_box(X0[p], Y0[p], W0[p], m0x1[p], m3x1[p], m6x1[p], cx, cy, X, Y);
        const uint32_t tX = X << 11, tY = Y << 11;
        const uint32_t cr = __builtin_amdgcn_perm(tY, tX, 0x07060302u);  // (column, row) as u16 x 2
        const uint32_t off = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, cr), pitch2, 0u, false);
        const uint16_t* t = reinterpret_cast<const uint16_t*>(sbytes + off);
        const uint32_t fx = X & 31, fy = Y & 31;
        const uint32_t v00 = t[0], v01 = t[1], v10 = t[box.pitch], v11 = t[box.pitch + 1];
        if constexpr (DARK) {
          const uint32_t ax = 32 - fx, ay = 32 - fy;
          uint32_t h0 = __umul24(v00, ax) + __umul24(v01, fx);
          uint32_t h1 = __umul24(v10, ax) + __umul24(v11, fx);
          asm volatile("" : "+v"(h0), "+v"(h1));  // keep the separable form (see output_rows)
          o[p] = round_q10(__umul24(h0, ay) + __umul24(h1, fy));
        } else {
          o[p] = blend_exact(v00, v01, v10, v11, (int)fx, (int)fy);
        }
        continue;
      }
      int X, Y;
      persp_px<MODE == 0>(X0[p], Y0[p], W0[p], m0x1[p], m3x1[p], m6x1[p], X, Y);
      if (MODE == 0) {
        const int fx = X & 31, fy = Y & 31;
        const int li = (int)__umul24((uint32_t)((Y >> 5) - box.sy0), (uint32_t)box.pitch) + ((X >> 5) - box.ax0);
#pragma unroll
        for (int k = 0; k < C; ++k) {
          const int i00 = li * C + k, i10 = i00 + box.pitch * C;
          o[p * C + k] = blend_exact(tap(stile, i00), tap(stile, i00 + C), tap(stile, i10), tap(stile, i10 + C), fx, fy);
        }
      } else if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < C; ++k) o[p * C + k] = 0;
      } else {
        bilinear_px<C>(S, H, W, X, Y, o + p * C);
      }
    }
    uint16_t* drow = Dst + ((size_t)y * W + x) * C;
    if (pair_store) {
      // streaming store: the aligned frame is written once and not re-read by this kernel
      __builtin_nontemporal_store((uint32_t)o[0] | ((uint32_t)o[1] << 16), reinterpret_cast<uint32_t*>(drow));
    } else if (C >= 3 && x + 2 <= W) {
      // two whole pixels: 6 (RGB) or 8 (RGBA) channels as 4-byte stores (x even -> aligned)
#pragma unroll
      for (int k = 0; k < C; ++k)
        __builtin_nontemporal_store((uint32_t)o[2 * k] | ((uint32_t)o[2 * k + 1] << 16),
                                    reinterpret_cast<uint32_t*>(drow) + k);
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (x + q < W)
#pragma unroll
          for (int k = 0; k < C; ++k) drow[q * C + k] = o[q * C + k];
    }
  }
}

template <int C, class Cfg = BlockCfg>
__global__ __launch_bounds__(kThreads) __attribute__((target("no-unaligned-access-mode"))) void
warp_perspective_u16_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                            const TilePlan* __restrict__ plan, const double* __restrict__ minv, int H, int W, int bw0) {
  __shared__ __attribute__((aligned(16))) uint16_t stile[Cfg::kLdsElems];
  const int ntx = gridDim.x, nty = gridDim.y;
  const int tile = xcd_remap(blockIdx.x + ntx * (blockIdx.y + nty * blockIdx.z), ntx * nty * gridDim.z);
  const int f = tile / (ntx * nty);
  const int t2 = tile - f * ntx * nty;
  const int xb = (t2 % ntx) * kTileW, yb = (t2 / ntx) * Cfg::kTileH;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const uint16_t* S = src + (size_t)f * H * W * C;
  uint16_t* Dst = dst + (size_t)f * H * W * C;

  const Box box = unpack(plan[tile]);
  KCMC_LDS_SENTINEL(stile, Cfg::kLdsElems, tid);
  const bool vec_stage = (C == 1) && ((W & 7) == 0);
  uint4 chunk[Cfg::kRowPasses];
  uint4 cchunk[C > 1 ? VecC<Cfg, C>::kPasses : 1];
  if (box.mode == 0 && vec_stage) stage_issue<Cfg>(S, box, H, W, tid, chunk);
  if constexpr (C > 1) {
    if (box.mode == 0 && (W & 7) == 0) stage_vec_c_issue<Cfg, C>(S, box, H, W, tid, cchunk);
  }
  double M[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) M[k] = minv[9 * (size_t)f + k];
  double* ptab = reinterpret_cast<double*>(stile + PerspTab<Cfg>::kBoxElems);
  const bool tab = bw0 == 64 && box.mode != 1;  // uniform
  if (tab) {
    for (int e = tid; e < PerspTab<Cfg>::kEntries; e += kThreads) {
      const double dy = (double)(yb + (e >> 1)), dxo = (double)(xb + 64 * (e & 1));
      ptab[3 * e] = M[0] * dxo + M[1] * dy + M[2];
      ptab[3 * e + 1] = M[3] * dxo + M[4] * dy + M[5];
      ptab[3 * e + 2] = M[6] * dxo + M[7] * dy + M[8];
    }
  }
  uint32_t* flags = reinterpret_cast<uint32_t*>(stile) + PerspTab<Cfg>::kFlagWord;
  if (box.mode == 0) {
    if (vec_stage) {
      stage_land<Cfg>(stile, box, tid, chunk);
      // bright (>= 16384) staged chunks of the box, counted per wave into the flag words
      uint32_t nb = 0;
#pragma unroll
      for (int k = 0; k < Cfg::kRowPasses; ++k)
        nb += __builtin_popcountll(
            __builtin_amdgcn_ballot_w64(((chunk[k].x | chunk[k].y | chunk[k].z | chunk[k].w) & 0xc000c000u) != 0));
      if (lane == 0) flags[wave] = nb;
    } else if (C > 1 && (W & 7) == 0) {
      if constexpr (C > 1) stage_vec_c_land<Cfg, C>(stile, box, tid, cchunk);
    } else
      stage_scalar<C>(S, stile, box, H, W, tid);
  }
  __syncthreads();
  if (box.mode == 1)
    persp_rows<Cfg, C, 1, false>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
  else if (tab) {
    if (box.mode == 0) {
      const uint4 fl = *reinterpret_cast<const uint4*>(flags);
      if (vec_stage && fl.x + fl.y + fl.z + fl.w == 0)
        persp_rows<Cfg, C, 0, true, true>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
      else
        persp_rows<Cfg, C, 0, true>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
    } else
      persp_rows<Cfg, C, 2, true>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
  } else if (box.mode == 0) {
    persp_rows<Cfg, C, 0, false>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
  } else {
    persp_rows<Cfg, C, 2, false>(stile, box, S, Dst, M, H, W, xb, yb, wave, lane, bw0, ptab);
  }
}

template <class Cfg>
size_t persp_workspace_bytes(int n_frames, int H, int W) {
  const size_t tiles = (size_t)ceil_div(W, kTileW) * ceil_div(H, Cfg::kTileH) * n_frames;
  return tiles * sizeof(TilePlan) + (size_t)n_frames * 9 * sizeof(double);
}

// WarpPerspectiveInvoker's block width: bh0 = min(16, H), bw0 = min(1024 / bh0, W)
inline int persp_bw0(int H, int W) {
  const int bh0 = H < 16 ? H : 16;
  return 1024 / bh0 < W ? 1024 / bh0 : W;
}

// Workspace layout of the perspective warp: minv [F, 9] f64, plan [tiles].
template <int C, class Cfg = typename CfgFor<C>::type>
void launch_persp_plan(const double* M, int n_frames, int H, int W, int inverse_map, void* ws, hipStream_t s) {
  const int ntx = ceil_div(W, kTileW), nty = ceil_div(H, Cfg::kTileH);
  const long long tiles = (long long)ntx * nty * n_frames;
  double* minv = static_cast<double*>(ws);
  TilePlan* plan = reinterpret_cast<TilePlan*>(minv + 9 * (size_t)n_frames);
  hipLaunchKernelGGL((persp_plan_kernel<C, Cfg>), dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, s, M, n_frames,
                     H, W, inverse_map, ntx, nty, plan, minv);
}

template <int C, class Cfg = typename CfgFor<C>::type>
void launch_persp_tiles(const uint16_t* src, uint16_t* dst, int n_frames, int H, int W, const void* ws, hipStream_t s) {
  const int ntx = ceil_div(W, kTileW), nty = ceil_div(H, Cfg::kTileH);
  const double* minv = static_cast<const double*>(ws);
  const TilePlan* plan = reinterpret_cast<const TilePlan*>(minv + 9 * (size_t)n_frames);
  hipLaunchKernelGGL((warp_perspective_u16_kernel<C, Cfg>), dim3(ntx, nty, n_frames), dim3(kThreads), 0, s, src, dst,
                     plan, minv, H, W, persp_bw0(H, W));
}

template <int C, class Cfg = typename CfgFor<C>::type>
void launch_persp(const uint16_t* src, uint16_t* dst, const double* M, int n_frames, int H, int W, int inverse_map,
                  void* ws, hipStream_t s) {
  launch_persp_plan<C, Cfg>(M, n_frames, H, W, inverse_map, ws, s);
  launch_persp_tiles<C, Cfg>(src, dst, n_frames, H, W, ws, s);
}

// The plan workspace of one warp call (both launch forms use the same layout).
size_t plan_bytes(int n_frames, int H, int W, int C, bool perspective) {
  if (perspective)
    return C == 1 ? persp_workspace_bytes<BlockCfg>(n_frames, H, W) : persp_workspace_bytes<ChanCfg>(n_frames, H, W);
  if (C == 1) return use_tile64(H) ? warp_workspace_bytes<Block64Cfg>(n_frames, H, W)
                                   : warp_workspace_bytes<BlockCfg>(n_frames, H, W);
  return warp_workspace_bytes<ChanCfg>(n_frames, H, W);
}

// The plan / tile launches of a warp call; `tiles` false: the plan, true: the tiles.
void launch_part(bool tiles, bool perspective, const uint16_t* src, uint16_t* dst, const double* M, int n_frames,
                 int H, int W, int C, int inverse_map, void* ws, hipStream_t s) {
  if (perspective) {
    switch (C) {
      case 1:
        tiles ? launch_persp_tiles<1>(src, dst, n_frames, H, W, ws, s)
              : launch_persp_plan<1>(M, n_frames, H, W, inverse_map, ws, s);
        break;
      case 3:
        tiles ? launch_persp_tiles<3>(src, dst, n_frames, H, W, ws, s)
              : launch_persp_plan<3>(M, n_frames, H, W, inverse_map, ws, s);
        break;
      default:
        tiles ? launch_persp_tiles<4>(src, dst, n_frames, H, W, ws, s)
              : launch_persp_plan<4>(M, n_frames, H, W, inverse_map, ws, s);
        break;
    }
    return;
  }
  switch (C) {
    case 1:
      if (use_tile64(H))
        tiles ? launch_warp_tiles<1, Block64Cfg>(src, dst, n_frames, H, W, ws, s)
              : launch_warp_plan<1, Block64Cfg>(M, n_frames, H, W, inverse_map, ws, s);
      else
        tiles ? launch_warp_tiles<1>(src, dst, n_frames, H, W, ws, s)
              : launch_warp_plan<1>(M, n_frames, H, W, inverse_map, ws, s);
      break;
    case 3:
      tiles ? launch_warp_tiles<3>(src, dst, n_frames, H, W, ws, s)
            : launch_warp_plan<3>(M, n_frames, H, W, inverse_map, ws, s);
      break;
    default:
      tiles ? launch_warp_tiles<4>(src, dst, n_frames, H, W, ws, s)
            : launch_warp_plan<4>(M, n_frames, H, W, inverse_map, ws, s);
      break;
  }
}

// The argument checks shared by every warp entry point.
int check_warp_args(const char* who, int n_frames, int H, int W, int C) {
  const std::string w(who);
  if (n_frames < 0 || H < 0 || W < 0) return fail(KCMC_EINVAL, w + ": negative size");
  if (H > 32767 || W > 32767) return fail(KCMC_EUNSUPPORTED, w + ": H, W must be < 32768");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, w + ": at most 65535 frames per call");
  if (C != 1 && C != 3 && C != 4) return fail(KCMC_EUNSUPPORTED, w + ": C must be 1, 3 or 4");
  if ((long long)ceil_div(W, kTileW) * ceil_div(H, ChanCfg::kTileH) * n_frames >= (1ll << 31))
    return fail(KCMC_EUNSUPPORTED, w + ": too many tiles in one call");
  return KCMC_OK;
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_warp_perspective_u16(kcmc_ctx* ctx, const uint16_t* src, uint16_t* dst, const double* M,
                                         int n_frames, int H, int W, int C, int inverse_map, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_warp_perspective_u16: ctx is NULL");
  KCMC_TRY(check_warp_args("kcmc_warp_perspective_u16", n_frames, H, W, C));
  if (n_frames == 0 || H == 0 || W == 0) return KCMC_OK;
  if (!src || !dst || !M) return fail(KCMC_EINVAL, "kcmc_warp_perspective_u16: NULL pointer");
  if (src == dst) return fail(KCMC_EINVAL, "kcmc_warp_perspective_u16: in-place warp is not supported");
  hipStream_t s = (hipStream_t)stream;
  void* ws = nullptr;
  const size_t wsb = plan_bytes(n_frames, H, W, C, true);
  KCMC_TRY(workspace_alloc(ctx, &ws, wsb, s));
  launch_part(false, true, src, dst, M, n_frames, H, W, C, inverse_map, ws, s);
  launch_part(true, true, src, dst, M, n_frames, H, W, C, inverse_map, ws, s);
  const int rc = launch_check("warp_perspective_u16_kernel");
  KCMC_TRY(workspace_free(ctx, ws, s, wsb));
  return rc;
}

extern "C" int kcmc_warp_affine_u16(kcmc_ctx* ctx, const uint16_t* src, uint16_t* dst, const double* M,
                                    int n_frames, int H, int W, int C, int inverse_map, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: ctx is NULL");
  KCMC_TRY(check_warp_args("kcmc_warp_affine_u16", n_frames, H, W, C));
  if (n_frames == 0 || H == 0 || W == 0) return KCMC_OK;
  if (!src || !dst || !M) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: NULL pointer");
  if (src == dst) return fail(KCMC_EINVAL, "kcmc_warp_affine_u16: in-place warp is not supported");
  hipStream_t s = (hipStream_t)stream;
  void* ws = nullptr;
  const size_t wsb = plan_bytes(n_frames, H, W, C, false);
  KCMC_TRY(workspace_alloc(ctx, &ws, wsb, s));
  launch_part(false, false, src, dst, M, n_frames, H, W, C, inverse_map, ws, s);
  launch_part(true, false, src, dst, M, n_frames, H, W, C, inverse_map, ws, s);
  const int rc = launch_check("warp_affine_u16_kernel");
  KCMC_TRY(workspace_free(ctx, ws, s, wsb));
  return rc;
}
