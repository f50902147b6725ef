// K1f: batched k=2 L2 matching of float32 descriptors (SIFT-style, BASELINE config 5).
//
// The reference matches uint8 AKAZE/BRISK descriptors (VA:194-195, match.hip); config 5
// asks for float descriptors, where the distance is a genuine dense fp32 contraction.
// Distance definition (OpenCV's batchDistL2_32f accumulates in a
// build-dependent SIMD order, so parity with it is unpinned): the near-exact
//   S = sum_k ((double)a_k - (double)b_k)^2 (sequential, fp64), dist = sqrtf((float)S),
// top-2 by (dist, frame index) like OpenCV's K-insertion.
//
// Phase 1 finds, per template row, a short candidate list on the fp16 matrix cores with a
// certified error bound; phase 2 ranks the candidates with the exact definition.
//
// tpl_stats_kernel / tpl_err_kernel -- once per call: K = max |a|^2 over the template
//   rows, the largest |a_k| (its power-of-2 scale s_T maps it into (2^14, 2^15]) and the
//   largest norm of a row's fp16 rounding error.
//
// frame_images_kernel -- one workgroup per 64-row tile: the exact LDS image the matcher
//   copies (18 KiB: fp16(s_f b) rows padded to 272 B, s_f = s_T / 2^8, then per row
//   C' = s_T s_f ((|b|^2 + K) / 2 + beta_j)); rows past the frame's last: zeros and
//   C' = +inf; and the frame's max |b|^2 and max beta_j.
//
// knn2_l2f32_kernel -- one workgroup = 256 template rows x one frame (8 waves x one block
//   of 32 rows, the template operand fp16(-s_T a) in registers).  Tiles reach LDS by
//   LDS-DMA (two buffers: one tile in flight ahead of the one in use, one barrier per
//   tile; 36 KB, so three workgroups = 6 waves per SIMD fit a CU).  One v_mfma_f32_32x32x16_f16 per 16-wide k-step and 32-row half tile, the
//   accumulator started at C':
//     v~ = s_T s_f ((|b|^2 + K) / 2 + beta_j - a.b + e_j),  |e_j| <= beta_j
//   (fp16 products are exact in fp32; e_j = the fp16 roundings of a and b, the fp32
//   accumulation and the norms, bounded below at its use), so v~ orders a lane's frame
//   rows like |a - b|^2 = 2 v + |a|^2 - K up to 2 beta, and v~ >= 0.  A distance costs a
//   compare with the list's bound and, when some lane of the wave needs it, 9 VALU: the
//   key (v~'s bits with the low bits replaced by the frame row: 1 op), a sorted top-8
//   insertion (v_med3_u32 x 7 + v_min_u32).  After the frame, the top-8 of
//   the two lane halves are merged; when the 8th value exceeds v(2) (1 + 2T) + 2B the
//   exact top-2 lies among the listed rows below that bound (usually 2-3), which phase 2
//   re-evaluates with the exact fp64 definition and orders by (dist, index).  Rows that
//   cannot be certified (8+ rows within 2B of the second) are appended to their frame's
//   list, which knn2_l2f32_fallback_kernel finishes by exact brute force.
#include <cfloat>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

typedef float v16f __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kBlk = 1;                   // 32-row template blocks per wave (2 measured slower)
constexpr int kThreads = 512 / kBlk;
constexpr int kWaves = kThreads / 64;
constexpr int kWavesPerEU = 6;            // occupancy target (register budget 512 / it)
constexpr int kNBuf = 2;                  // tile buffers: one tile in flight ahead of the one in use
constexpr int kTplPerWG = kWaves * 32 * kBlk;  // 256 template rows per workgroup
constexpr int kDP = 128;                  // padded descriptor length
constexpr int kKSteps = kDP / 16;         // k-steps of v_mfma_f32_32x32x16_f16
constexpr int kTile = 64;                 // frame rows per tile image (two MFMA row blocks)
constexpr int kRowB = kDP + 8;            // padded LDS row (fp16 elements, 272 B)
constexpr int kImgC = kTile * kRowB * 2;  // byte offset of the per-row C' values
constexpr int kImgBytes = 18 * 1024;      // tile image, whole 1 KiB LDS-DMA pieces
constexpr int kPieces = kImgBytes / 1024;
static_assert(kImgC + kTile * 4 <= kImgBytes, "tile image layout");
constexpr int kTop = 8;                   // approximate top-K per lane
// frame_images_kernel: rows per 16-lane group (4, 256-thread workgroups: faster alone,
// slower in the c5 step)
constexpr int kImgRows = 1;
constexpr int kImgThreads = kTile * 16 / kImgRows;  // threads per 64-row tile

// The build's exact distance (identical operation order in the oracle).
__device__ __forceinline__ float exact_dist(const float* __restrict__ a, const float* __restrict__ b, int D) {
  double S = 0.0;
  for (int k = 0; k < D; ++k) {
    const double t = (double)a[k] - (double)b[k];
    S += t * t;
  }
  return sqrtf((float)S);
}

// The same sum for 16-byte aligned rows with D % 4 == 0, read four floats per load.
__device__ __forceinline__ float exact_dist4(const float* __restrict__ a, const float* __restrict__ b, int D) {
  double S = 0.0;
  for (int k = 0; k < D; k += 4) {
    const float4 x = *reinterpret_cast<const float4*>(a + k), y = *reinterpret_cast<const float4*>(b + k);
    double t = (double)x.x - (double)y.x;
    S += t * t;
    t = (double)x.y - (double)y.y;
    S += t * t;
    t = (double)x.z - (double)y.z;
    S += t * t;
    t = (double)x.w - (double)y.w;
    S += t * t;
  }
  return sqrtf((float)S);
}

__device__ __forceinline__ float exact_dist_any(const float* __restrict__ a, const float* __restrict__ b, int D) {
  const bool v4 = (D & 3) == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
  return v4 ? exact_dist4(a, b, D) : exact_dist(a, b, D);
}

// (dist, index) lexicographic order: OpenCV's insertion gives ties to the lower index.
__device__ __forceinline__ bool lex_less(float d, int j, float e, int k) { return d < e || (d == e && j < k); }

__device__ __forceinline__ void top2_insert_exact(float& d0, int& j0, float& d1, int& j1, float d, int j) {
  if (lex_less(d, j, d0, j0)) {
    d1 = d0;
    j1 = j0;
    d0 = d;
    j0 = j;
  } else if (lex_less(d, j, d1, j1)) {
    d1 = d;
    j1 = j;
  }
}

// Workgroups are dealt round-robin over the 8 XCDs: give each XCD a contiguous run of
// ids (bijective also when n % 8 != 0).
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int q8 = n >> 3, r8 = n & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Sorted top-kTop of 32-bit keys (k0 <= k1 <= ...): kTop VALU per insertion.
__device__ __forceinline__ void topk_key(uint32_t (&k)[kTop], uint32_t x) {
#pragma unroll
  for (int i = kTop - 1; i > 0; --i) k[i] = med3_u32(k[i - 1], k[i], x);
  k[0] = min(k[0], x);
}

// One distance of the tile loop: if its value bits x are below the list's last key k7
// (some lane of the wave takes the branch), key = (x & kmask) | id enters the sorted top-8
// in place (v_and_or_b32 + 7 v_med3_u32 + v_min_u32: 9 VALU).  Comparing the raw bits with
// k7 keeps the bound the certification needs: a rejected x >= k7 truncates to >= the last
// listed value, and so does every key the list pushes out.  Hand-written because the
// backend gave the updated list fresh registers on every insertion and copied it back
// (6-10 v_mov per insertion); id is wave-uniform (an SGPR), kmask a VGPR (a VOP3 reads
// one SGPR at most).
// AFTER_MFMA: x was written by the MFMA just issued; hipcc pads nothing inside an asm
// string, so the string opens with the 12 wait states an 8-pass XDL result needs before a
// VALU reads it (the later values of the tile are read more than 12 states later).
#define KCMC_TOPK_TRY_BODY                             \
  "v_cmp_lt_u32 vcc, %[x], %[k7]\n\t"                  \
  "s_and_saveexec_b64 %[sv], vcc\n\t"                  \
  "s_cbranch_execz 1f\n\t"                             \
  "v_and_or_b32 %[x], %[x], %[km], %[id]\n\t"          \
  "v_med3_u32 %[k7], %[k6], %[k7], %[x]\n\t"           \
  "v_med3_u32 %[k6], %[k5], %[k6], %[x]\n\t"           \
  "v_med3_u32 %[k5], %[k4], %[k5], %[x]\n\t"           \
  "v_med3_u32 %[k4], %[k3], %[k4], %[x]\n\t"           \
  "v_med3_u32 %[k3], %[k2], %[k3], %[x]\n\t"           \
  "v_med3_u32 %[k2], %[k1], %[k2], %[x]\n\t"           \
  "v_med3_u32 %[k1], %[k0], %[k1], %[x]\n\t"           \
  "v_min_u32 %[k0], %[k0], %[x]\n"                      \
  "1:\n\t"                                             \
  "s_or_b64 exec, exec, %[sv]"
#define KCMC_TOPK_TRY_OPERANDS                                                                                 \
  : [k0] "+v"(k[0]), [k1] "+v"(k[1]), [k2] "+v"(k[2]), [k3] "+v"(k[3]), [k4] "+v"(k[4]), [k5] "+v"(k[5]),      \
    [k6] "+v"(k[6]), [k7] "+v"(k[7]), [x] "+v"(xb), [sv] "=&s"(saved)                                         \
  : [km] "v"(kmask), [id] "s"(id)                                                                             \
  : "vcc"
template <bool AFTER_MFMA>
__device__ __forceinline__ void topk_try(uint32_t (&k)[kTop], uint32_t xb, uint32_t kmask, uint32_t id) {
  static_assert(kTop == 8, "topk_try keeps a top-8");
  uint64_t saved;
  if constexpr (AFTER_MFMA)
    asm volatile("s_nop 11\n\t" KCMC_TOPK_TRY_BODY KCMC_TOPK_TRY_OPERANDS);
  else
    asm volatile(KCMC_TOPK_TRY_BODY KCMC_TOPK_TRY_OPERANDS);
}
#undef KCMC_TOPK_TRY_BODY
#undef KCMC_TOPK_TRY_OPERANDS

// Sorted approximate top-kTop values with the frame rows of the first kTop - 1.
struct TopK {
  float v[kTop];
  int j[kTop - 1];
};

__device__ __forceinline__ void topk_insert(TopK& t, float x, int j) {
  bool c[kTop];
#pragma unroll
  for (int i = 0; i < kTop; ++i) c[i] = x < t.v[i];
  t.v[kTop - 1] = c[kTop - 2] ? t.v[kTop - 2] : (c[kTop - 1] ? x : t.v[kTop - 1]);
#pragma unroll
  for (int i = kTop - 2; i > 0; --i) {
    t.v[i] = c[i - 1] ? t.v[i - 1] : (c[i] ? x : t.v[i]);
    t.j[i] = c[i - 1] ? t.j[i - 1] : (c[i] ? j : t.j[i]);
  }
  t.v[0] = c[0] ? x : t.v[0];
  t.j[0] = c[0] ? j : t.j[0];
}

// Power-of-2 scale that maps a largest magnitude m into (2^14, 2^15]: fp16 then holds every
// scaled value (max 65504) with 11 significant bits; 1 for m == 0 / non-finite m, clamped
// to [2^-60, 2^60] (a frame outside that range is certified nowhere and falls back).
__device__ __forceinline__ float pow2_scale(float m) {
  if (!(m > 0.f) || !(m < INFINITY)) return 1.f;
  int e;
  (void)frexpf(m, &e);  // m < 2^e
  return ldexpf(1.f, max(-60, min(60, 15 - e)));
}

// Bias of row j's accumulator start (unscaled units): beta_j >= |e_j| for every template
// row, e_j the phase-1 error of v~_j.  With a'' = fp16(s_T a) / s_T = a - da and b'' = b -
// db the values the matrix cores multiply (fp16 products are exact in fp32):
// |a.b - a''.b''| <= |da||b| + |a||db| + |da||db|, where |da| <= dA (the template's
// largest rounding-error norm, tpl_err_kernel) and |db_j| is the row's own (both computed
// from the actual roundings, subnormals included); the fp32 accumulation of C' and D
// products (rounding or truncating) <= (D + 1) 2u 1.01 S_j with S_j <= U_j / 2 + beta_j,
// U_j = (sqrt(K) + |b_j|)^2, u = 2^-24; the norm, K, halving, bias and scaling roundings
// <= (D + 4) u U_j / 2; K below an exact |a|^2 by <= D u K / 2.  Sum <= dA |b_j| +
// sqrt(K) |db_j| (1 + 2^-10) + (3.6 D + 6) u U_j; taken as 1.1 (dA |b| + sqrt(K) |db| +
// (4 D + 8) u U).  (|a| <= sqrt(K) (1 + D u / 2), |b_j| <= sqrt(ss_j) (1 + D u) and the
// fp32 evaluation of the norms are inside the 1.1.)
__device__ __forceinline__ float beta_of(float sK, float nb, float dA, float db, int D) {
  const float U = (sK + nb) * (sK + nb);
  return 1.1f * (dA * nb + sK * db + (float)(4 * D + 8) * 5.9604645e-8f * U) + 1e-30f;
}

constexpr int kTplRowsPerWG = 64;  // tpl_stats_kernel / tpl_err_kernel: 8 row groups x 8 rows

// Workgroup max of a non-negative float (bits) -> one atomicMax.
__device__ __forceinline__ void wg_atomic_max(float v, unsigned* dst) {
  __shared__ float s_w[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(dst, __float_as_uint(fmaxf(fmaxf(s_w[0], s_w[1]), fmaxf(s_w[2], s_w[3]))));
}

// Kst[0] = K = max_i |a_i|^2, Kst[1] = max |a_ik| (non-negative float bits, zeroed before
// the launch).  32 lanes per row, 4 floats each; 8 rows per 32-lane group.
__global__ __launch_bounds__(256) void tpl_stats_kernel(const float* __restrict__ des_tpl, int n_tpl, int D,
                                                        unsigned* __restrict__ Kst) {
  const int col = (threadIdx.x & 31) * 4;
  float K = 0.f, mx = 0.f;
  for (int rr = 0; rr < 8; ++rr) {
    const int i = blockIdx.x * kTplRowsPerWG + (threadIdx.x >> 5) * 8 + rr;
    if (i >= n_tpl) break;  // whole 32-lane groups together
    const float* src = des_tpl + (size_t)i * D;
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (col + k < D) {
        ss = fmaf(src[col + k], src[col + k], ss);
        mx = fmaxf(mx, fabsf(src[col + k]));
      }
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    K = fmaxf(K, ss);
  }
  wg_atomic_max(K, &Kst[0]);
  wg_atomic_max(mx, &Kst[1]);
}

// Kst[2] = dA >= max_i |a_i - fp16(s_T a_i) / s_T| (fp64 sums, rounded up): the
// template's largest rounding-error norm on the matrix cores.
__global__ __launch_bounds__(256) void tpl_err_kernel(const float* __restrict__ des_tpl, int n_tpl, int D,
                                                      unsigned* __restrict__ Kst) {
  const float sT = pow2_scale(__uint_as_float(Kst[1]));
  const int col = (threadIdx.x & 31) * 4;
  float dA = 0.f;
  for (int rr = 0; rr < 8; ++rr) {
    const int i = blockIdx.x * kTplRowsPerWG + (threadIdx.x >> 5) * 8 + rr;
    if (i >= n_tpl) break;  // whole 32-lane groups together
    const float* src = des_tpl + (size_t)i * D;
    double e2 = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (col + k < D) {
        const double d = (double)src[col + k] - (double)(float)(_Float16)(src[col + k] * sT) / (double)sT;
        e2 += d * d;
      }
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) e2 += __shfl_xor(e2, off);
    dA = fmaxf(dA, (float)(sqrt(e2) * 1.000001) + 1e-38f);
  }
  wg_atomic_max(dA, &Kst[2]);
}

// Tile t of frame f -> img[(f * tpf + t) * kImgBytes]: fp16(s_f b) rows with s_f = s_T /
// 2^8 (frame values up to 2^8 x the template's largest element are in range; smaller ones
// keep 11 bits down to 2^-14 and the subnormal rest is in |db|), per row C'; and the
// frame's max |b|^2 / max beta_j (fmax / fbeta, zeroed before the launch).  A value
// beyond fp16's range flags the frame (fbad), whose rows are then all certified nowhere
// (exact fallback).  One workgroup per tile: 16 lanes per row, 8 elements each, kImgRows rows
// per lane group with all their loads issued before the first conversion.
__device__ __forceinline__ float frame_scale(const unsigned* __restrict__ Kst) {
  return pow2_scale(__uint_as_float(Kst[1])) * 0.00390625f;
}

__global__ __launch_bounds__(kImgThreads) void frame_images_kernel(const float* __restrict__ des_q, int D,
                                                                   const int32_t* __restrict__ q_off, int tpf,
                                                                   const unsigned* __restrict__ Kst,
                                                                   uint8_t* __restrict__ img,
                                                                   unsigned* __restrict__ fmax,
                                                                   unsigned* __restrict__ fbeta,
                                                                   int32_t* __restrict__ fbad) {
  constexpr int kGroups = kImgThreads / 16;  // 16-lane row groups; group g owns rows g, g + kGroups, ...
  const int t = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const int q_begin = q_off[f];
  const int n_q = min(q_off[f + 1] - q_begin, tpf * kTile);
  if (t * kTile >= n_q) return;  // the whole workgroup
  const float* base = des_q + (size_t)q_begin * D;
  const bool v4 = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(base) & 15) == 0;
  const float K = __uint_as_float(Kst[0]);
  const float sK = sqrtf(K);
  const float sT = pow2_scale(__uint_as_float(Kst[1]));
  const float sf = frame_scale(Kst);
  const float isf = 1.f / sf;  // exact: s_f is a power of 2 in [2^-68, 2^52]
  const float sc = sT * sf;
  const float dA = __uint_as_float(Kst[2]);
  const int g = tid >> 4, col = (tid & 15) * 8;
  uint8_t* tile = img + ((size_t)f * tpf + t) * kImgBytes;
  // every row's loads first (kImgRows rows per lane in flight), then the conversions
  float x[kImgRows][8];
#pragma unroll
  for (int i = 0; i < kImgRows; ++i) {
    const int r = t * kTile + g + i * kGroups;
#pragma unroll
    for (int k = 0; k < 8; ++k) x[i][k] = 0.f;
    if (r < n_q) {
      const float* src = base + (size_t)r * D;
      if (v4) {
        if (col < D) {
          const float4 p = *reinterpret_cast<const float4*>(src + col);
          x[i][0] = p.x; x[i][1] = p.y; x[i][2] = p.z; x[i][3] = p.w;
        }
        if (col + 4 < D) {
          const float4 p = *reinterpret_cast<const float4*>(src + col + 4);
          x[i][4] = p.x; x[i][5] = p.y; x[i][6] = p.z; x[i][7] = p.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[i][k] = col + k < D ? src[col + k] : 0.f;
      }
    }
  }
  float nmax = 0.f, bmax = 0.f;
  bool big = false;
#pragma unroll
  for (int i = 0; i < kImgRows; ++i) {
    const int rr = g + i * kGroups;
    const bool real = t * kTile + rr < n_q;
    float ss = 0.f, e2 = 0.f;
    f16x8 h;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ss = fmaf(x[i][k], x[i][k], ss);
      const float y = x[i][k] * sf;
      big |= !(fabsf(y) <= 65504.f);  // also NaN
      h[k] = (_Float16)y;
      const float d = x[i][k] - (float)h[k] * isf;  // the rounding error, exact (isf = 1 / s_f, a power of 2)
      e2 = fmaf(d, d, e2);
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
      ss += __shfl_xor(ss, off);
      e2 += __shfl_xor(e2, off);
    }
    *reinterpret_cast<f16x8*>(tile + (rr * kRowB + col) * 2) = h;
    if ((tid & 15) == 15)  // the row's 16 bytes of padding: every image line is written whole
      *reinterpret_cast<uint4*>(tile + (rr * kRowB + kDP) * 2) = make_uint4(0u, 0u, 0u, 0u);
    if ((tid & 15) == 0) {
      const float beta = beta_of(sK, sqrtf(ss), dA, sqrtf(e2), D);
      *reinterpret_cast<float*>(tile + kImgC + 4 * rr) = real ? (0.5f * (ss + K) + beta) * sc : INFINITY;
      if (real) {
        nmax = fmaxf(nmax, ss);
        bmax = fmaxf(bmax, beta);
      }
    }
  }
  static_assert((kImgBytes - kImgC - kTile * 4) / 16 <= kImgThreads, "image tail");
  if (tid < (kImgBytes - kImgC - kTile * 4) / 16)  // the image's tail after the C' values
    *reinterpret_cast<uint4*>(tile + kImgC + kTile * 4 + 16 * tid) = make_uint4(0u, 0u, 0u, 0u);
  if (__any(big) && (tid & 63) == 0) atomicOr(&fbad[f], 1);
  __shared__ float s_n[kImgThreads / 64], s_b[kImgThreads / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    nmax = fmaxf(nmax, __shfl_xor(nmax, off));
    bmax = fmaxf(bmax, __shfl_xor(bmax, off));
  }
  if ((tid & 63) == 0) {
    s_n[tid >> 6] = nmax;
    s_b[tid >> 6] = bmax;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kImgThreads / 64; ++w) {
      nmax = fmaxf(nmax, s_n[w]);
      bmax = fmaxf(bmax, s_b[w]);
    }
    atomicMax(&fmax[f], __float_as_uint(nmax));
    atomicMax(&fbeta[f], __float_as_uint(bmax));
  }
}

// One tile image (18 x 1 KiB) global -> LDS: wave w copies pieces w, w + kWaves, ...
// (each lane 16 B; the LDS destination of a piece is M0 + lane * 16).  Issued by inline
// asm: with __builtin_amdgcn_global_load_lds the compiler treats every later ds_read of
// the staging array as dependent on every copy in flight and waits vmcnt(0) before it,
// which drains the prefetch; here the counted vmcnt waits and the barrier in the tile
// loop order the copies against the reads (M0 is saved and restored around each issue).
__device__ __forceinline__ void dma_piece(const uint8_t* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}
__device__ __forceinline__ void dma_tile(const uint8_t* __restrict__ src, uint8_t* dst, int wave, int lane) {
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(dst);  // the LDS offset
#pragma unroll
  for (int p0 = 0; p0 < kPieces; p0 += kWaves) {
    const int p = p0 + wave;  // wave-uniform
    if (p < kPieces)
      dma_piece(src + p * 1024 + lane * 16, (uint32_t)__builtin_amdgcn_readfirstlane((int)(base + (uint32_t)(p * 1024))));
  }
}

// Decode, merge, certify and re-rank one template row i of the wave (the lane's list ck).
__device__ __forceinline__ void finish_row(const uint32_t (&ck)[kTop], int i, int c, int h, int f, int n_tpl, int D,
                                           const float* __restrict__ des_tpl, const float* __restrict__ des_q,
                                           int q_begin, int n_q, const unsigned* __restrict__ Kst,
                                           const float* __restrict__ fmax, const float* __restrict__ fbeta,
                                           const int32_t* __restrict__ fbad, int key_bits, uint32_t kmask,
                                           int32_t* __restrict__ out_idx, float* __restrict__ out_dist,
                                           int32_t* __restrict__ fallback, int32_t* __restrict__ fb_cnt,
                                           int32_t* __restrict__ fb_frames, unsigned long long* __restrict__ fb_keys) {
  const float sT = pow2_scale(__uint_as_float(Kst[1]));
  // ---- decode (value truncated to the key, frame row) and merge the two row halves
  // (lanes c and c + 32 own the same template row)
  TopK best;
#pragma unroll
  for (int k = 0; k < kTop; ++k) {
    const uint32_t low = ck[k] & ~kmask;
    best.v[k] = ck[k] == 0xffffffffu ? INFINITY : __uint_as_float(ck[k] & kmask);
    if (k < kTop - 1) {
      const int r = (int)(low & 15);
      best.j[k] = (int)(low >> 5) * kTile + (int)((low >> 4) & 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    }
  }
  {
    float ov[kTop];
    int oj[kTop - 1];
#pragma unroll
    for (int k = 0; k < kTop; ++k) ov[k] = __shfl_xor(best.v[k], 32);
#pragma unroll
    for (int k = 0; k < kTop - 1; ++k) oj[k] = __shfl_xor(best.j[k], 32);
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < kTop - 1; ++k) topk_insert(best, ov[k], oj[k]);
      // the partner's last value bounds every row it did not report
      best.v[kTop - 1] = fminf(best.v[kTop - 1], ov[kTop - 1]);
    }
    // the merged list to both halves: they share the exact re-rank below
#pragma unroll
    for (int k = 0; k < kTop; ++k) best.v[k] = __shfl(best.v[k], c, 64);
#pragma unroll
    for (int k = 0; k < kTop - 1; ++k) best.j[k] = __shfl(best.j[k], c, 64);
  }
  if (i >= n_tpl) return;

  // ---- certify and re-rank with the exact distance.  In scaled units (sc = s_T s_f):
  // v~_j is in [sc v_j, sc (v_j + 2B)] with B = max_j beta_j (fbeta), and a listed
  // value tv_j (a key: low key_bits bits cleared, relative truncation T <= 2^(key_bits - 23))
  // is in [v~_j (1 - T), v~_j].  An unlisted row has sc v_j >= tv_j - 2 sc B >= tv(6) -
  // 2 sc B, a listed one sc v_j <= tv_j / (1 - T): rows whose tv exceeds thr = tv(2) (1 + 2T)
  // + 2 sc B cannot reach the exact top-2 (the fp64 distance keeps the order of v up to
  // its rounding, far inside T).  A frame whose scaled values could overflow is not
  // certified (fallback).
  const float K = __uint_as_float(Kst[0]);
  const float sK = sqrtf(K);
  const float sc = sT * frame_scale(Kst);
  const float maxb = sqrtf(fmax[f]);
  const float Bs = fbeta[f] * sc;
  const float T = ldexpf(1.f, key_bits - 23);
  const float thr = best.v[1] * (1.f + 2.f * T) + 2.f * Bs;
  const bool sane = fbad[f] == 0 && sc * (K + maxb * maxb) < 1e36f && Bs < 1e36f;
  // (sanity first: a flagged frame's fp16 images overflow, and its values -- inf / NaN --
  // must not read as "fewer than two frame rows"; round 5, tests/test_gpu_fuzz.py)
  int ncand;
  if (!sane) {
    ncand = -1;
  } else if (!(best.v[1] < INFINITY)) {
    ncand = best.v[0] < INFINITY ? 1 : 0;  // fewer than two frame rows: all are listed
  } else if (!(best.v[kTop - 1] > thr)) {
    ncand = -1;
  } else {
    ncand = 2;
#pragma unroll
    for (int k = 2; k < kTop - 1; ++k) ncand += best.v[k] <= thr ? 1 : 0;
  }
  const size_t o = ((size_t)f * n_tpl + i) * 2;
  if (ncand < 0) {  // frame f's list (room for every template row)
    if (h != 0) return;
    const int slot = atomicAdd(&fb_cnt[f], 1);
    fallback[(size_t)f * n_tpl + slot] = i;
    fb_keys[2 * ((size_t)f * n_tpl + slot)] = ~0ull;  // the merge keys of the entry start empty
    fb_keys[2 * ((size_t)f * n_tpl + slot) + 1] = ~0ull;
    if (slot == 0) fb_frames[1 + atomicAdd(&fb_frames[0], 1)] = f;  // the frame's first entry lists it
    return;
  }
  // the candidates' exact distances, shared by the two lanes of the row: lane half h takes
  // candidates 2m + h (one pass for the usual two candidates instead of two)
  float d0 = FLT_MAX, d1 = FLT_MAX;
  int j0 = -1, j1 = -1;
  const float* a = des_tpl + (size_t)i * D;
  const float* fb = des_q + (size_t)q_begin * D;
#pragma unroll
  for (int m = 0; 2 * m < kTop - 1; ++m) {
    const int k = 2 * m + h;
    int j = best.j[2 * m];
    if (2 * m + 1 < kTop - 1 && h) j = best.j[2 * m + 1];
    if (k < ncand && (unsigned)j < (unsigned)n_q)  // (always in range; the guard keeps reads inside the frame)
      top2_insert_exact(d0, j0, d1, j1, exact_dist_any(a, fb + (size_t)j * D, D), j);
  }
  {
    const float e0 = __shfl_xor(d0, 32), e1 = __shfl_xor(d1, 32);
    const int k0 = __shfl_xor(j0, 32), k1 = __shfl_xor(j1, 32);
    if (k0 >= 0) top2_insert_exact(d0, j0, d1, j1, e0, k0);
    if (k1 >= 0) top2_insert_exact(d0, j0, d1, j1, e1, k1);
  }
  if (h != 0) return;
  out_idx[o] = j0;
  out_idx[o + 1] = j1;
  out_dist[o] = d0;
  out_dist[o + 1] = d1;
}

// 6 waves per SIMD (<= 80 VGPRs; the epilogue spills a few, the tile loop none): the
// waits on LDS and the MFMA results hide behind the other waves' top-K VALU work
// (c5 lab 4.56 -> 4.38 ms against 4 waves per SIMD with three tile buffers)
// (kBlk = 1; with kBlk = 2 a wave holds two template blocks, one LDS fragment read feeds two
// MFMAs, at 3 waves per SIMD)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kWavesPerEU, kWavesPerEU)))
void knn2_l2f32_kernel(
    const float* __restrict__ des_tpl, int n_tpl, int D, const float* __restrict__ des_q,
    const int32_t* __restrict__ q_off, const uint8_t* __restrict__ img, int tpf,
    const unsigned* __restrict__ Kst, const float* __restrict__ fmax, const float* __restrict__ fbeta,
    const int32_t* __restrict__ fbad, int key_bits, int32_t* __restrict__ out_idx, float* __restrict__ out_dist,
    int32_t* __restrict__ fallback, int32_t* __restrict__ fb_cnt, int32_t* __restrict__ fb_frames,
    unsigned long long* __restrict__ fb_keys) {
  __shared__ __attribute__((aligned(16))) uint8_t tbuf[kNBuf][kImgBytes];

  // XCD-aware order: the workgroups of one frame get consecutive ids of one XCD's run
  // (dispatch is round-robin over the 8 XCDs), so the frame's tile images stay in that
  // XCD's L2 for all of its template blocks
  const int ntb = gridDim.x;
  const int wg = xcd_remap(blockIdx.x + ntb * blockIdx.y, ntb * gridDim.y);
  const int f = wg / ntb, tb = wg - f * ntb;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31;  // MFMA column = template row within the wave's block
  const int h = lane >> 5;  // k-half of the fragments / row group of the output
  const int q_begin = q_off[f];
  const int n_q = q_off[f + 1] - q_begin;
  const int n_tiles = min((n_q + kTile - 1) / kTile, tpf);
  const uint8_t* fimg = img + (size_t)f * tpf * kImgBytes;
  if (n_tiles > 0) dma_tile(fimg, tbuf[0], wave, lane);

  // ---- template fragment (B operand, fp16(-s_T a)) kept in registers: lane (c, h) holds
  // row i's elements k = 16 s + 8 h + j of k-step s
  const float sT = pow2_scale(__uint_as_float(Kst[1]));
  const int i0 = tb * kTplPerWG + wave * 32 * kBlk + c;  // block b: row i0 + 32 b
  f16x8 btpl[kBlk][kKSteps];
#pragma unroll
  for (int b = 0; b < kBlk; ++b)
#pragma unroll
    for (int st = 0; st < kKSteps; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 32 * b, k = 16 * st + 8 * h + j;
        const float v = (i < n_tpl && k < D) ? des_tpl[(size_t)i * D + k] : 0.f;
        btpl[b][st][j] = (_Float16)(-v * sT);
      }

  // keys: v~'s bits with the low key_bits bits replaced by (tile << 5 | half << 4 | r)
  const uint32_t kmask = ~((1u << key_bits) - 1u);
  uint32_t ck[kBlk][kTop];
#pragma unroll
  for (int b = 0; b < kBlk; ++b)
#pragma unroll
    for (int k = 0; k < kTop; ++k) ck[b][k] = 0xffffffffu;
  int cur = 0;  // t % kNBuf
  for (int t = 0; t < n_tiles; ++t) {
    // tile t has landed (this wave's pieces: vmcnt; the others': the barrier) and every
    // wave is done with tile t - 1, whose buffer the copy of tile t + 1 overwrites.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < n_tiles) dma_tile(fimg + (size_t)(t + 1) * kImgBytes, tbuf[cur ^ 1], wave, lane);
    const uint8_t* tbp = tbuf[cur];
    cur ^= 1;
    // accumulators start at the rows' C': half hh, lane's 16 rows 32 hh + (r & 3) + 8 (r >> 2) + 4h
    const float* cq = reinterpret_cast<const float*>(tbp + kImgC);
    const uint32_t tbase = (uint32_t)t << 5;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      v16f acc[kBlk];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 q4 = *reinterpret_cast<const float4*>(cq + 32 * hh + 8 * g + 4 * h);
#pragma unroll
        for (int b = 0; b < kBlk; ++b) {
          acc[b][4 * g] = q4.x;
          acc[b][4 * g + 1] = q4.y;
          acc[b][4 * g + 2] = q4.z;
          acc[b][4 * g + 3] = q4.w;
        }
      }
      const _Float16* ap = reinterpret_cast<const _Float16*>(tbp) + (32 * hh + c) * kRowB + 8 * h;
      // one LDS fragment read feeds every block's MFMA
#pragma unroll
      for (int st = 0; st < kKSteps; ++st) {
        const f16x8 av = *reinterpret_cast<const f16x8*>(ap + 16 * st);
#pragma unroll
        for (int b = 0; b < kBlk; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, btpl[b][st], acc[b], 0, 0, 0);
      }
      // a value whose bits are >= the last key cannot enter the list (its truncation is >=
      // the last listed value, which already bounds every unlisted row).  After the first
      // few hundred rows most distances of a wave skip the insertion (the branch is per
      // wave): 1 + 7 P VALU per distance, P = the share of the wave's values some lane
      // inserts (0.31 on the c5 data, simulated; 0.34 from the round-3 PMC's INT32 count)
#pragma unroll
      for (int b = 0; b < kBlk; ++b) {
        topk_try<true>(ck[b], __float_as_uint(acc[b][0]), kmask, (uint32_t)(hh * 16) | tbase);
#pragma unroll
        for (int r = 1; r < 16; ++r)
          topk_try<false>(ck[b], __float_as_uint(acc[b][r]), kmask, (uint32_t)(hh * 16 + r) | tbase);
      }
    }
  }
#pragma unroll
  for (int b = 0; b < kBlk; ++b)
    finish_row(ck[b], i0 + 32 * b, c, h, f, n_tpl, D, des_tpl, des_q, q_begin, n_q, Kst, fmax, fbeta, fbad, key_bits,
               kmask, out_idx, out_dist, fallback, fb_cnt, fb_frames, fb_keys);
}


// Exact brute force for the rows phase 1 could not certify: frame f's listed template
// rows (fb[f * n_tpl + k], k < fb_cnt[f]) in batches of up to kFbBatch.  Workgroup
// (f, y, z) scans slice y of the frame's rows for batches z, z + kFbLanes, ... (so a
// frame with a few listed rows still spreads over kFbSplit workgroups, and one with many
// over kFbSplit x kFbLanes); each distance is one lane's sequential
// fp64 sum (the build's definition), then a wave-wide and a workgroup-wide lexicographic
// top-2 merge per listed row, and the slices' top-2 meet in two 64-bit keys per listed
// row, (dist bits << 32 | index) -- u64 order is the (dist, index) order -- through
// atomicMin: the key that loses at the first slot (max(old, new)) goes to the second,
// so the second slot ends as the smallest key that ever lost = the second smallest.
// knn2_l2f32_fallback_out_kernel writes the results.
constexpr int kFbThreads = 256;
constexpr int kFbBatch = 4;
constexpr int kFbSplit = 16;  // frame-row slices per frame
constexpr int kFbLanes = 4;   // batch lanes: workgroup (f, y, z) takes batches z, z + kFbLanes, ...

template <int NB>
__device__ __forceinline__ void fb_scan(const float (*sa)[kDP], const float* __restrict__ frame, int j_lo, int j_hi,
                                        int D, bool v4, int tid, float (&d0)[kFbBatch], int (&j0)[kFbBatch],
                                        float (&d1)[kFbBatch], int (&j1)[kFbBatch]) {
  for (int j = j_lo + tid; j < j_hi; j += kFbThreads) {
    const float* row = frame + (size_t)j * D;
    double S[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) S[b] = 0.0;
    if (v4) {
      // unrolled so that the loads of several pieces of the row are in flight together
      // (one lane walks a whole row: each load is its own cache line)
#pragma unroll 8
      for (int k = 0; k < D; k += 4) {
        const float4 y = *reinterpret_cast<const float4*>(row + k);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float4 x = *reinterpret_cast<const float4*>(&sa[b][k]);
          double t = (double)x.x - (double)y.x;
          S[b] += t * t;
          t = (double)x.y - (double)y.y;
          S[b] += t * t;
          t = (double)x.z - (double)y.z;
          S[b] += t * t;
          t = (double)x.w - (double)y.w;
          S[b] += t * t;
        }
      }
    } else {
      for (int k = 0; k < D; ++k) {
        const double y = (double)row[k];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const double t = (double)sa[b][k] - y;
          S[b] += t * t;
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) top2_insert_exact(d0[b], j0[b], d1[b], j1[b], sqrtf((float)S[b]), j);
  }
}

__device__ __forceinline__ unsigned long long fb_key(float d, int j) {
  return ((unsigned long long)__float_as_uint(d) << 32) | (uint32_t)j;
}

__global__ __launch_bounds__(kFbThreads) void knn2_l2f32_fallback_kernel(const float* __restrict__ des_tpl, int n_tpl,
                                                                         int D, const float* __restrict__ des_q,
                                                                         const int32_t* __restrict__ q_off,
                                                                         const int32_t* __restrict__ fb,
                                                                         const int32_t* __restrict__ fb_cnt,
                                                                         const int32_t* __restrict__ fb_frames,
                                                                         unsigned long long* __restrict__ fb_keys) {
  __shared__ __attribute__((aligned(16))) float sa[kFbBatch][kDP];
  __shared__ float sd[kFbThreads / 64][kFbBatch][2];
  __shared__ int sj[kFbThreads / 64][kFbBatch][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool v4 = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(des_q) & 15) == 0;
  // work items (listed frame, slice y, batch lane z), grid-stride: only the frames with
  // listed rows are visited (a grid over every frame launched ~32k mostly idle workgroups)
  const int n_items = fb_frames[0] * kFbSplit * kFbLanes;
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
  const int f = fb_frames[1 + item / (kFbSplit * kFbLanes)];
  const int y = (item / kFbLanes) % kFbSplit, z = item % kFbLanes;
  const int cnt = fb_cnt[f];
  const int q_begin = q_off[f], n_q = q_off[f + 1] - q_begin;
  const int j_lo = (int)((long long)n_q * y / kFbSplit);
  const int j_hi = (int)((long long)n_q * (y + 1) / kFbSplit);
  for (int k0 = z * kFbBatch; k0 < cnt; k0 += kFbLanes * kFbBatch) {
    const int nb = min(kFbBatch, cnt - k0);
    __syncthreads();  // the previous batch's merge is done with sa / sd / sj
    for (int e = tid; e < kFbBatch * kDP; e += kFbThreads) {
      const int b = e / kDP, k = e - b * kDP;
      sa[b][k] = (b < nb && k < D) ? des_tpl[(size_t)fb[(size_t)f * n_tpl + k0 + b] * D + k] : 0.f;
    }
    __syncthreads();
    float d0[kFbBatch], d1[kFbBatch];
    int j0[kFbBatch], j1[kFbBatch];
#pragma unroll
    for (int b = 0; b < kFbBatch; ++b) {
      d0[b] = d1[b] = FLT_MAX;
      j0[b] = j1[b] = -1;
    }
    const float* frame = des_q + (size_t)q_begin * D;
    switch (nb) {  // workgroup-uniform
      case 1: fb_scan<1>(sa, frame, j_lo, j_hi, D, v4, tid, d0, j0, d1, j1); break;
      case 2: fb_scan<2>(sa, frame, j_lo, j_hi, D, v4, tid, d0, j0, d1, j1); break;
      case 3: fb_scan<3>(sa, frame, j_lo, j_hi, D, v4, tid, d0, j0, d1, j1); break;
      default: fb_scan<4>(sa, frame, j_lo, j_hi, D, v4, tid, d0, j0, d1, j1); break;
    }
#pragma unroll
    for (int b = 0; b < kFbBatch; ++b) {
      for (int off = 32; off > 0; off >>= 1) {
        const float e0 = __shfl_xor(d0[b], off), e1 = __shfl_xor(d1[b], off);
        const int m0 = __shfl_xor(j0[b], off), m1 = __shfl_xor(j1[b], off);
        if (m0 >= 0) top2_insert_exact(d0[b], j0[b], d1[b], j1[b], e0, m0);
        if (m1 >= 0) top2_insert_exact(d0[b], j0[b], d1[b], j1[b], e1, m1);
      }
      if (lane == 0) {
        sd[wave][b][0] = d0[b];
        sd[wave][b][1] = d1[b];
        sj[wave][b][0] = j0[b];
        sj[wave][b][1] = j1[b];
      }
    }
    __syncthreads();
    if (tid < nb) {
      const int b = tid;
      float e0 = sd[0][b][0], e1 = sd[0][b][1];
      int m0 = sj[0][b][0], m1 = sj[0][b][1];
      for (int v = 1; v < kFbThreads / 64; ++v)
        for (int k = 0; k < 2; ++k)
          if (sj[v][b][k] >= 0) top2_insert_exact(e0, m0, e1, m1, sd[v][b][k], sj[v][b][k]);
      unsigned long long* key = fb_keys + 2 * ((size_t)f * n_tpl + k0 + b);
      if (m0 >= 0) {
        const unsigned long long k = fb_key(e0, m0);
        const unsigned long long o = atomicMin(&key[0], k);
        atomicMin(&key[1], o > k ? o : k);
      }
      if (m1 >= 0) {
        const unsigned long long k = fb_key(e1, m1);
        const unsigned long long o = atomicMin(&key[0], k);
        atomicMin(&key[1], o > k ? o : k);
      }
    }
  }
  }
}

// The listed rows' merged keys -> out_idx / out_dist (no key: index -1, FLT_MAX); one
// workgroup per listed frame, grid-stride.
__global__ __launch_bounds__(256) void knn2_l2f32_fallback_out_kernel(int n_tpl, const int32_t* __restrict__ fb,
                                                                      const int32_t* __restrict__ fb_cnt,
                                                                      const int32_t* __restrict__ fb_frames,
                                                                      const unsigned long long* __restrict__ fb_keys,
                                                                      int32_t* __restrict__ out_idx,
                                                                      float* __restrict__ out_dist) {
  for (int q = blockIdx.x; q < fb_frames[0]; q += gridDim.x) {
    const int f = fb_frames[1 + q];
    const int cnt = fb_cnt[f];
    for (int k = threadIdx.x; k < cnt; k += 256) {
      const size_t slot = (size_t)f * n_tpl + k;
      const size_t o = ((size_t)f * n_tpl + fb[slot]) * 2;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const unsigned long long key = fb_keys[2 * slot + r];
        const bool ok = key != ~0ull;
        out_idx[o + r] = ok ? (int32_t)(uint32_t)key : -1;
        out_dist[o + r] = ok ? __uint_as_float((uint32_t)(key >> 32)) : FLT_MAX;
      }
    }
  }
}

int check_f32_args(const void* des_tpl, int n_tpl, int D, const void* des_q, const void* q_off, int n_frames,
                   int max_nq, const void* o1, const void* o2) {
  if (n_tpl < 0 || n_frames < 0 || max_nq < 0) return fail(KCMC_EINVAL, "match_f32: negative size");
  if (D < 1 || D > kDP)
    return fail(KCMC_EUNSUPPORTED, "match_f32: descriptor length D must be in [1, 128] (got " + std::to_string(D) + ")");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "match_f32: at most 65535 frames per call");
  if ((long long)n_frames * n_tpl >= (1ll << 31)) return fail(KCMC_EUNSUPPORTED, "match_f32: n_frames * n_tpl too large");
  if (n_frames > 0 && n_tpl > 0 && (!des_tpl || !q_off || !o1 || !o2 || (max_nq > 0 && !des_q)))
    return fail(KCMC_EINVAL, "match_f32: NULL pointer");
  return KCMC_OK;
}

// Layout of the two work areas of a float match.  The prepared part (template stats,
// the frames' max |b|^2 / max beta / bad flags, then the tile images: tpf = ceil(max_nq /
// 64) per frame; the CSR total is a device value); the run part holds the per-frame fallback
// counters, the listed frames (count + ids) and lists (room for every template row) and
// the fallback merge keys (set by the matcher when it lists a row).
struct F32Layout {
  int tpf = 0, key_bits = 0;
  size_t stat_bytes = 0, img_bytes = 0, cnt_bytes = 0, fb_bytes = 0, key_bytes = 0;
  size_t prep_bytes() const { return stat_bytes + img_bytes; }
  size_t run_bytes() const { return cnt_bytes + fb_bytes + key_bytes; }
};

F32Layout f32_layout(int n_tpl, int n_frames, int max_nq) {
  F32Layout L;
  const size_t rows = (size_t)n_frames * n_tpl;
  L.tpf = ceil_div(max(max_nq, 0), kTile);
  int tbits = 0;
  while ((1 << tbits) < L.tpf) ++tbits;
  L.key_bits = 5 + tbits;  // (tile << 5 | half << 4 | register)
  L.stat_bytes = (256 + 3 * (size_t)n_frames * sizeof(float) + 255) & ~(size_t)255;
  L.img_bytes = (size_t)n_frames * L.tpf * kImgBytes;
  L.cnt_bytes = ((2 * (size_t)n_frames + 1) * sizeof(int32_t) + 255) & ~(size_t)255;
  L.fb_bytes = (rows * sizeof(int32_t) + 255) & ~(size_t)255;
  L.key_bytes = rows * 2 * sizeof(unsigned long long);
  return L;
}

// The prepared part: template stats, then the frames' tile images and stats.
int launch_f32_prepare(const F32Layout& L, const float* des_tpl, int n_tpl, int D, const float* des_q,
                       const int32_t* q_off, int n_frames, void* prep, hipStream_t s) {
  char* w = static_cast<char*>(prep);
  unsigned* Kst = reinterpret_cast<unsigned*>(w);
  unsigned* fmax = reinterpret_cast<unsigned*>(w + 256);  // max |b|^2, max beta, bad flag
  unsigned* fbeta = fmax + n_frames;
  int32_t* fbad = reinterpret_cast<int32_t*>(fbeta + n_frames);
  uint8_t* img = reinterpret_cast<uint8_t*>(w + L.stat_bytes);
  KCMC_TRY(hip_check(hipMemsetAsync(Kst, 0, L.stat_bytes, s), "hipMemsetAsync"));
  hipLaunchKernelGGL(tpl_stats_kernel, dim3(ceil_div(n_tpl, kTplRowsPerWG)), dim3(256), 0, s, des_tpl, n_tpl, D, Kst);
  KCMC_TRY(launch_check("tpl_stats_kernel"));
  hipLaunchKernelGGL(tpl_err_kernel, dim3(ceil_div(n_tpl, kTplRowsPerWG)), dim3(256), 0, s, des_tpl, n_tpl, D, Kst);
  KCMC_TRY(launch_check("tpl_err_kernel"));
  if (L.tpf > 0) {
    hipLaunchKernelGGL(frame_images_kernel, dim3(L.tpf, n_frames), dim3(kImgThreads), 0, s, des_q, D, q_off, L.tpf,
                       Kst, img, fmax, fbeta, fbad);
    KCMC_TRY(launch_check("frame_images_kernel"));
  }
  return KCMC_OK;
}

// The matcher and its exact fallback on a prepared part.
int launch_f32_run(const F32Layout& L, const float* des_tpl, int n_tpl, int D, const float* des_q,
                   const int32_t* q_off, int n_frames, const void* prep, void* run, int32_t* out_idx, float* out_dist,
                   hipStream_t s) {
  const char* w = static_cast<const char*>(prep);
  const unsigned* Kst = reinterpret_cast<const unsigned*>(w);
  const unsigned* fmax = reinterpret_cast<const unsigned*>(w + 256);
  const unsigned* fbeta = fmax + n_frames;
  const int32_t* fbad = reinterpret_cast<const int32_t*>(fbeta + n_frames);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(w + L.stat_bytes);
  char* r = static_cast<char*>(run);
  int32_t* fb_cnt = reinterpret_cast<int32_t*>(r);
  int32_t* fb = reinterpret_cast<int32_t*>(r + L.cnt_bytes);
  unsigned long long* fb_keys = reinterpret_cast<unsigned long long*>(r + L.cnt_bytes + L.fb_bytes);
  int32_t* fb_frames = fb_cnt + n_frames;
  KCMC_TRY(hip_check(hipMemsetAsync(fb_cnt, 0, (size_t)(n_frames + 1) * sizeof(int32_t), s), "hipMemsetAsync"));
  hipLaunchKernelGGL(knn2_l2f32_kernel, dim3(ceil_div(n_tpl, kTplPerWG), n_frames), dim3(kThreads), 0, s, des_tpl,
                     n_tpl, D, des_q, q_off, img, L.tpf, Kst, reinterpret_cast<const float*>(fmax),
                     reinterpret_cast<const float*>(fbeta), fbad, L.key_bits, out_idx, out_dist, fb, fb_cnt, fb_frames,
                     fb_keys);
  KCMC_TRY(launch_check("knn2_l2f32_kernel"));
  const int fb_grid = min(n_frames * kFbSplit * kFbLanes, 4 * device_cus());
  hipLaunchKernelGGL(knn2_l2f32_fallback_kernel, dim3(fb_grid), dim3(kFbThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off,
                     fb, fb_cnt, fb_frames, fb_keys);
  KCMC_TRY(launch_check("knn2_l2f32_fallback_kernel"));
  hipLaunchKernelGGL(knn2_l2f32_fallback_out_kernel, dim3(min(n_frames, 1024)), dim3(256), 0, s, n_tpl, fb, fb_cnt,
                     fb_frames, fb_keys, out_idx, out_dist);
  return launch_check("knn2_l2f32_fallback_out_kernel");
}

int f32_layout_check(const F32Layout& L) {
  if (L.key_bits > 20) return fail(KCMC_EUNSUPPORTED, "match_f32: more than 2^21 descriptors in one frame");
  return KCMC_OK;
}

// Both parts in one stream-ordered workspace.
int launch_knn_f32(kcmc_ctx* ctx, const float* des_tpl, int n_tpl, int D, const float* des_q, const int32_t* q_off,
                   int n_frames, int max_nq, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  const F32Layout L = f32_layout(n_tpl, n_frames, max_nq);
  KCMC_TRY(f32_layout_check(L));
  const size_t own = L.prep_bytes();
  void* ws = nullptr;
  KCMC_TRY(workspace_alloc(ctx, &ws, own + L.run_bytes(), s));
  char* w = static_cast<char*>(ws);
  int rc = launch_f32_prepare(L, des_tpl, n_tpl, D, des_q, q_off, n_frames, w, s);
  if (rc == KCMC_OK) rc = launch_f32_run(L, des_tpl, n_tpl, D, des_q, q_off, n_frames, w, w + own, out_idx, out_dist, s);
  const int rf = workspace_free(ctx, ws, s);
  return rc != KCMC_OK ? rc : rf;
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_knn2_l2f32(kcmc_ctx* ctx, const float* des_tpl, int n_tpl, int D, const float* des_q,
                               const int32_t* q_off, int n_frames, int max_nq, int32_t* out_idx, float* out_dist,
                               kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_knn2_l2f32: ctx is NULL");
  KCMC_TRY(check_f32_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  return launch_knn_f32(ctx, des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist, (hipStream_t)stream);
}

extern "C" int kcmc_match_frames_f32(kcmc_ctx* ctx, const float* des_tpl, const double* kp_tpl, int n_tpl, int D,
                                     const float* des_q, const double* kp_q, const int32_t* q_off, int n_frames,
                                     int max_nq, double ratio, double d_lo, double d_hi, int32_t* out_idx,
                                     float* out_dist, double* out_kp_ordered, uint32_t* out_keep_bits,
                                     int32_t* out_counts, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_match_frames_f32: ctx is NULL");
  KCMC_TRY(check_f32_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  if (n_frames > 0 && n_tpl > 0 && (!kp_tpl || !out_kp_ordered || !out_keep_bits || !out_counts || (max_nq > 0 && !kp_q)))
    return fail(KCMC_EINVAL, "kcmc_match_frames_f32: NULL pointer");
  if (n_tpl > 8192) return fail(KCMC_EUNSUPPORTED, "kcmc_match_frames_f32: n_tpl > 8192");
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  hipStream_t s = (hipStream_t)stream;
  KCMC_TRY(launch_knn_f32(ctx, des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist, s));
  return launch_match_filter(out_idx, out_dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio, d_lo, d_hi,
                             out_kp_ordered, out_keep_bits, out_counts, s);
}
