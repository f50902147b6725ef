// K1f: batched k=2 L2 matching of float32 descriptors (SIFT-style, BASELINE config 5).
//
// The reference matches uint8 AKAZE/BRISK descriptors (VA:194-195, match.hip); config 5
// asks for float descriptors, where the distance is a genuine dense fp32 contraction.
// Distance definition (OpenCV's batchDistL2_32f accumulates in a
// build-dependent SIMD order, so parity with it is unpinned): the near-exact
//   S = sum_k ((double)a_k - (double)b_k)^2 (sequential, fp64), dist = sqrtf((float)S),
// top-2 by (dist, frame index) like OpenCV's K-insertion.
//
// tpl_norm_max_kernel -- once per call: K = max over template rows of |a|^2 (fp32).
//
// split_tiles_kernel -- once per call: every frame's rows, 32 at a time, written as the
//   exact LDS image the matcher copies (18 KiB per tile: bf16 hi rows | bf16 lo rows, each
//   row padded to 272 B, then C = (|b|^2 + K) / 2 per row; v = hi + lo + e with
//   |e| <= 2^-18 |v|; hi = RNE(v), v - hi exact, lo = RNE(v - hi)), and each tile's
//   max |b|^2.  Rows past the frame's last get C = +inf.
//
// knn2_l2f32_kernel -- one workgroup = 256 template rows x one frame (8 waves x one block
//   of 32 rows).  Tiles reach LDS by LDS-DMA (global_load_lds_dwordx4, three buffers:
//   two tiles in flight ahead of the one in use, one barrier per tile; no staging
//   registers).  On the bf16 matrix cores, with the template
//   operand negated and the accumulator started at the row's C,
//     v = (|b|^2 + K) / 2 - a.b,  a.b ~ hi.hi + hi.lo + lo.hi
//   (v_mfma_f32_32x32x16_bf16, 3 MFMAs per k-step of 16: 5.3x fewer cycles than
//   v_mfma_f32_32x32x2_f32 for the same contraction).  v orders a lane's frame rows
//   exactly like |a - b|^2 = 2 v + |a|^2 - K (K >= |a|^2 keeps it non-negative), so a
//   distance costs 7 VALU: clamp, key (v's float bits with the low mantissa bits
//   replaced by the row within a group of kFoldTiles tiles), and the sorted top-4
//   insertion; each group's top-4 is folded into a running approximate top-4.  The
//   error of a listed value is bounded by
//     eps = (5 (D + 2) 2^-24 + 0.6 (3 2^-18 + t)) (sqrt(K) + max|b|)^2 * 1.02
//   with t = the keys' relative truncation (derivation at its use below).
//   (derivation at its use below).
//   A frame row can be among the exact top-2 only if v <= v(2) + 2 eps, so when the
//   approximate 4th value exceeds that bound the exact top-2 lies within the top-3
//   candidates: phase 2 re-evaluates them with the exact fp64 definition and orders
//   them by (dist, index).  Rows that cannot be certified (near-ties of 4+ frame
//   descriptors) are appended to their frame's list, which knn2_l2f32_fallback_kernel
//   finishes by exact brute force, reading each frame row once per batch of up to 4
//   listed rows.
#include <cfloat>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kNBuf = 3;                           // tile buffers: two tiles in flight ahead of the one in use
constexpr int kBlocks = 1;                         // 32-row template blocks per wave (2: 1 wave per SIMD)
constexpr int kTplPerWG = kWaves * kBlocks * 32;  // 256
constexpr int kDP = 128;                           // padded descriptor length
constexpr int kKSteps = kDP / 16;                  // k-steps of v_mfma_f32_32x32x16_bf16
constexpr int kTile = 32;                          // frame rows per tile image (one MFMA tile)
constexpr int kFoldTiles = 2;                      // tiles per top-4 fold (the row within them is in the key)
constexpr uint32_t kRowMask = kFoldTiles * kTile - 1;
// relative truncation of a key (its low log2(kFoldTiles * kTile) mantissa bits)
constexpr float kKeyTrunc = (float)(kFoldTiles * kTile) * 1.1920929e-7f;
constexpr int kRowB = kDP + 8;                     // padded LDS row (bf16 elements, 272 B)
constexpr int kImgLo = kTile * kRowB * 2;          // byte offset of the lo rows in a tile image
constexpr int kImgC = 2 * kImgLo;                  // byte offset of the per-row C values
constexpr int kImgBytes = 18 * 1024;               // tile image, whole 1 KiB LDS-DMA pieces
constexpr int kPieces = kImgBytes / 1024;
static_assert(kImgC + kTile * 4 <= kImgBytes, "tile image layout");
constexpr uint32_t kNoKey = 0xffffffffu;

// The build's exact distance (identical operation order in the oracle).
__device__ __forceinline__ float exact_dist(const float* __restrict__ a, const float* __restrict__ b, int D) {
  double S = 0.0;
  for (int k = 0; k < D; ++k) {
    const double t = (double)a[k] - (double)b[k];
    S += t * t;
  }
  return sqrtf((float)S);
}

// The same sum for 16-byte aligned rows with D % 4 == 0, read four floats per load (the
// fallback's lanes each walk a different frame row: a quarter of the load instructions).
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

// Approximate top-4 values (v0 <= v1 <= v2 <= v3) with the indices of the first three.
struct Top4 {
  float v[4];
  int j[3];
};

__device__ __forceinline__ void top4_insert(Top4& t, float x, int j) {
  const bool c0 = x < t.v[0], c1 = x < t.v[1], c2 = x < t.v[2], c3 = x < t.v[3];
  t.v[3] = c2 ? t.v[2] : (c3 ? x : t.v[3]);
  t.v[2] = c1 ? t.v[1] : (c2 ? x : t.v[2]);
  t.j[2] = c1 ? t.j[1] : (c2 ? j : t.j[2]);
  t.v[1] = c0 ? t.v[0] : (c1 ? x : t.v[1]);
  t.j[1] = c0 ? t.j[0] : (c1 ? j : t.j[1]);
  t.v[0] = c0 ? x : t.v[0];
  t.j[0] = c0 ? j : t.j[0];
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

// Sorted top-4 of 32-bit keys (k0 <= k1 <= k2 <= k3): 4 VALU per insertion.
__device__ __forceinline__ void top4_key(uint32_t (&k)[4], uint32_t x) {
  k[3] = med3_u32(k[2], k[3], x);
  k[2] = med3_u32(k[1], k[2], x);
  k[1] = med3_u32(k[0], k[1], x);
  k[0] = min(k[0], x);
}

// bf16 split of an fp32 value: v = hi + lo + e with |e| <= 2^-18 |v| (hi = RNE(v), the
// difference v - hi is exact in fp32, lo = RNE(v - hi)).
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

// K = max_i |a_i|^2 over the template rows (positive float bits order as integers; *Kbits
// zeroed before the launch).  32 lanes per row, 4 floats each.
__global__ __launch_bounds__(256) void tpl_norm_max_kernel(const float* __restrict__ des_tpl, int n_tpl, int D,
                                                           unsigned* __restrict__ Kbits) {
  const int i = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (i >= n_tpl) return;  // whole 32-lane groups exit together
  const int col = (threadIdx.x & 31) * 4;
  const float* src = des_tpl + (size_t)i * D;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (col + k < D) ss = fmaf(src[col + k], src[col + k], ss);
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
  if ((threadIdx.x & 31) == 0) atomicMax(Kbits, __float_as_uint(ss));
}

// Frame f's tile t (rows 32 t .. 32 t + 31) -> img[(f * tpf + t) * kImgBytes]: the LDS
// image the matcher copies (hi rows, lo rows, C = (|b|^2 + K) / 2 per row; rows past the
// frame's last: zero descriptors, C = +inf), and the tile's max |b|^2 -> tile_max[f * tpf
// + t].  One workgroup per tile, 8 rows per pass (32 lanes per row, 4 floats each).
__global__ __launch_bounds__(256) void split_tiles_kernel(const float* __restrict__ des_q, int D,
                                                          const int32_t* __restrict__ q_off, int tpf,
                                                          const unsigned* __restrict__ Kbits,
                                                          uint8_t* __restrict__ img,
                                                          float* __restrict__ tile_max) {
  __shared__ float s_max[4];
  const int f = blockIdx.y, t = blockIdx.x;
  const int n_q = q_off[f + 1] - q_off[f];
  const int n_rows = min(n_q, tpf * kTile);
  if (t * kTile >= n_rows) return;  // the whole workgroup
  const int col = (threadIdx.x & 31) * 4;
  const bool v4 = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(des_q) & 15) == 0;
  const float K = __uint_as_float(*Kbits);
  uint8_t* tile = img + ((size_t)f * tpf + t) * kImgBytes;
  float tmax = 0.f;
#pragma unroll
  for (int pass = 0; pass < kTile / 8; ++pass) {
    const int rr = pass * 8 + (threadIdx.x >> 5);
    const int r = t * kTile + rr;
    const bool real = r < n_rows;
    const float* src = des_q + (size_t)(q_off[f] + r) * D;
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (real) {
      if (v4) {
        if (col < D) w = *reinterpret_cast<const float4*>(src + col);
      } else {
        w.x = col < D ? src[col] : 0.f;
        w.y = col + 1 < D ? src[col + 1] : 0.f;
        w.z = col + 2 < D ? src[col + 2] : 0.f;
        w.w = col + 3 < D ? src[col + 3] : 0.f;
      }
    }
    float ss = fmaf(w.w, w.w, fmaf(w.z, w.z, fmaf(w.y, w.y, w.x * w.x)));
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    tmax = fmaxf(tmax, ss);
    if ((threadIdx.x & 31) == 0) *reinterpret_cast<float*>(tile + kImgC + 4 * rr) = real ? 0.5f * (ss + K) : INFINITY;
    __bf16 hv[4], lv[4];
    split_bf16(w.x, hv[0], lv[0]);
    split_bf16(w.y, hv[1], lv[1]);
    split_bf16(w.z, hv[2], lv[2]);
    split_bf16(w.w, hv[3], lv[3]);
    *reinterpret_cast<uint2*>(tile + (rr * kRowB + col) * 2) = *reinterpret_cast<const uint2*>(hv);
    *reinterpret_cast<uint2*>(tile + kImgLo + (rr * kRowB + col) * 2) = *reinterpret_cast<const uint2*>(lv);
    // the rows' padding columns too: every cache line of the image is written whole
    if (col == kDP - 4) {
      *reinterpret_cast<uint4*>(tile + (rr * kRowB + kDP) * 2) = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(tile + kImgLo + (rr * kRowB + kDP) * 2) = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  // and the image's tail after the C values
  for (int e = kImgC + kTile * 4 + 16 * (int)threadIdx.x; e < kImgBytes; e += 16 * 256)
    *reinterpret_cast<uint4*>(tile + e) = make_uint4(0u, 0u, 0u, 0u);
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
  if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = tmax;
  __syncthreads();
  if (threadIdx.x == 0)
    tile_max[(size_t)f * tpf + t] = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
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

// 4 waves per SIMD (<= 128 VGPRs): without the cap the compiler hoists every fragment
// read of a tile (239 VGPRs, 2 waves per SIMD)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void knn2_l2f32_kernel(
    const float* __restrict__ des_tpl, int n_tpl, int D, const float* __restrict__ des_q,
    const int32_t* __restrict__ q_off, const uint8_t* __restrict__ img, int tpf,
    const unsigned* __restrict__ Kbits, const float* __restrict__ tile_max, int32_t* __restrict__ out_idx,
    float* __restrict__ out_dist, int32_t* __restrict__ fallback, int32_t* __restrict__ fb_cnt) {
  __shared__ __attribute__((aligned(16))) uint8_t tbuf[kNBuf][kImgBytes];

  // XCD-aware order: the workgroups of one frame get consecutive ids of one XCD's run
  // (dispatch is round-robin over the 8 XCDs), so the frame's tile images stay in that
  // XCD's L2 for all of its template blocks
  const int ntb = gridDim.x;
  const int wg = xcd_remap(blockIdx.x + ntb * blockIdx.y, ntb * gridDim.y);
  const int f = wg / ntb, tb = wg - f * ntb;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31;  // MFMA column = template row within a block
  const int h = lane >> 5;  // k-half of the fragments / row group of the output
  const int q_begin = q_off[f];
  const int n_q = q_off[f + 1] - q_begin;
  const int n_tiles = min((n_q + kTile - 1) / kTile, tpf);
  const uint8_t* fimg = img + (size_t)f * tpf * kImgBytes;
  if (n_tiles > 0) dma_tile(fimg, tbuf[0], wave, lane);
  if (n_tiles > 1) dma_tile(fimg + kImgBytes, tbuf[1], wave, lane);
  // LDS-DMA pieces this wave issues per tile (wave-uniform): the count left in flight
  // while tile t + 1 is still landing
  const bool many = wave < kPieces % kWaves;
  static_assert(kPieces / kWaves == 2 && kPieces % kWaves != 0, "vmcnt counts below assume 2 or 3 pieces per wave");

  // ---- template fragments (B operand, bf16 hi/lo split of -a) kept in registers: lane
  // (c, h) holds row i's elements k = 16 s + 8 h + j of k-step s
  bf16x8 bhi[kBlocks][kKSteps], blo[kBlocks][kKSteps];
  int tpl_row[kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const int i = tb * kTplPerWG + (wave * kBlocks + b) * 32 + c;
    tpl_row[b] = i;
#pragma unroll
    for (int st = 0; st < kKSteps; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * st + 8 * h + j;
        const float v = (i < n_tpl && k < D) ? des_tpl[(size_t)i * D + k] : 0.f;
        __bf16 hv, lv;
        split_bf16(-v, hv, lv);
        bhi[b][st][j] = hv;
        blo[b][st][j] = lv;
      }
  }

  Top4 best[kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
#pragma unroll
    for (int k = 0; k < 4; ++k) best[b].v[k] = INFINITY;
#pragma unroll
    for (int k = 0; k < 3; ++k) best[b].j[k] = -1;
  }
  uint32_t ck[kBlocks][4];
  int cur = 0;  // t % kNBuf
  for (int t = 0; t < n_tiles; ++t) {
    // tile t has landed (this wave's pieces: vmcnt, leaving tile t + 1's in flight; the
    // others': the barrier) and every wave is done with tile t - 1, whose buffer the copy
    // of tile t + 2 overwrites.  A raw s_barrier: __syncthreads() would wait vmcnt(0).
    if (t + 1 == n_tiles)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (many)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < n_tiles) {
      const int nb = cur >= 1 ? cur - 1 : kNBuf - 1;  // (t + 2) % kNBuf
      dma_tile(fimg + (size_t)(t + 2) * kImgBytes, tbuf[nb], wave, lane);
    }
    const uint8_t* tbp = tbuf[cur];
    cur = cur + 1 == kNBuf ? 0 : cur + 1;
    if ((t & (kFoldTiles - 1)) == 0) {
#pragma unroll
      for (int b = 0; b < kBlocks; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k) ck[b][k] = kNoKey;
    }
    // accumulators start at the rows' C: lane's 16 rows (r & 3) + 8 (r >> 2) + 4h
    const float* cq = reinterpret_cast<const float*>(tbp + kImgC);
    v16f acc0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 q4 = *reinterpret_cast<const float4*>(cq + 8 * g + 4 * h);
      acc0[4 * g] = q4.x;
      acc0[4 * g + 1] = q4.y;
      acc0[4 * g + 2] = q4.z;
      acc0[4 * g + 3] = q4.w;
    }
    v16f acc[kBlocks];
#pragma unroll
    for (int b = 0; b < kBlocks; ++b) acc[b] = acc0;
    const __bf16* ah = reinterpret_cast<const __bf16*>(tbp) + c * kRowB + 8 * h;
    const __bf16* al = reinterpret_cast<const __bf16*>(tbp + kImgLo) + c * kRowB + 8 * h;
#pragma unroll
    for (int st = 0; st < kKSteps; ++st) {
      const bf16x8 a_h = *reinterpret_cast<const bf16x8*>(ah + 16 * st);
      const bf16x8 a_l = *reinterpret_cast<const bf16x8*>(al + 16 * st);
#pragma unroll
      for (int b = 0; b < kBlocks; ++b) {
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, bhi[b][st], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, blo[b][st], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, bhi[b][st], acc[b], 0, 0, 0);
      }
    }
    // keys: v's bits (negative v -> +0 by a signed max; +inf / NaN sort after every
    // finite key) with the row within the group of kFoldTiles tiles in the low bits
    const uint32_t pair_row = (uint32_t)(t & (kFoldTiles - 1)) * kTile + 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t row = pair_row + (uint32_t)((r & 3) + 8 * (r >> 2));
#pragma unroll
      for (int b = 0; b < kBlocks; ++b)
        top4_key(ck[b], ((uint32_t)max(__float_as_int(acc[b][r]), 0) & ~kRowMask) | row);
    }
    // ---- fold the group's top-4 into the running top-4 (the group's 4th key bounds
    // every row of the group it did not report, and so does the running 4th value)
    if ((t & (kFoldTiles - 1)) == kFoldTiles - 1 || t + 1 == n_tiles) {
      const int base = (t & ~(kFoldTiles - 1)) * kTile;
#pragma unroll
      for (int b = 0; b < kBlocks; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (ck[b][k] != kNoKey)
            top4_insert(best[b], __uint_as_float(ck[b][k] & ~kRowMask), base + (int)(ck[b][k] & kRowMask));
    }
  }
  // the frame's max |b|^2, from its tiles'
  float maxqn = 0.f;
  for (int t = lane; t < n_tiles; t += 64) maxqn = fmaxf(maxqn, tile_max[(size_t)f * tpf + t]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) maxqn = fmaxf(maxqn, __shfl_xor(maxqn, off));
  const float maxb = sqrtf(maxqn);
  const float sK = sqrtf(__uint_as_float(*Kbits));

  // ---- merge the two row halves (lanes c and c + 32 own the same template row)
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    float ov[4];
    int oj[3];
#pragma unroll
    for (int k = 0; k < 4; ++k) ov[k] = __shfl_xor(best[b].v[k], 32);
#pragma unroll
    for (int k = 0; k < 3; ++k) oj[k] = __shfl_xor(best[b].j[k], 32);
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) top4_insert(best[b], ov[k], oj[k]);
      // the partner's 4th value bounds every index it did not report
      best[b].v[3] = fminf(best[b].v[3], ov[3]);
    }
  }
  if (h != 0) return;

  // ---- certify and re-rank with the exact distance
  const float* base = des_q + (size_t)q_begin * D;
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const int i = tpl_row[b];
    if (i >= n_tpl) continue;
    const Top4& t = best[b];
    // |v~ - v| for every listed value, with v = (|b|^2 + K)/2 - a.b exact and
    // S = (|b|^2 + K)/2 + |a||b| <= U/2, U = (sqrt(K) + max|b|)^2, u = 2^-24: the norm and
    // C roundings (D + 1) u S; the bf16x3 residual 3 2^-18 S; the fp32 accumulation of
    // C and 3D exact bf16 products (rounding or truncating) (3D + 1) 2u 1.01 S; the key
    // truncation kKeyTrunc S.  Sum <= (4 (D + 1) u + (3 2^-18 + kKeyTrunc) / 2) U, taken
    // with margin as (5 (D + 2) u + 0.6 (3 2^-18 + kKeyTrunc)) U 1.02.
    const float U = (sK + maxb) * (sK + maxb);
    const float eps =
        (5.f * (float)(D + 2) * 5.9604645e-8f + 0.6f * (1.1444092e-5f + kKeyTrunc)) * U * 1.02f + 1e-30f;
    const float thr = t.v[1] + 2.f * eps;
    int ncand;
    if (!(t.v[1] < INFINITY)) {
      ncand = t.v[0] < INFINITY ? 1 : 0;  // fewer than two frame rows: all are listed
    } else if (t.v[2] > thr) {
      ncand = 2;
    } else if (t.v[3] > thr) {
      ncand = 3;
    } else {
      ncand = -1;
    }
    const size_t o = ((size_t)f * n_tpl + i) * 2;
    if (ncand < 0) {  // frame f's list (room for every template row)
      const int slot = atomicAdd(&fb_cnt[f], 1);
      fallback[(size_t)f * n_tpl + slot] = i;
      continue;
    }
    float d0 = FLT_MAX, d1 = FLT_MAX;
    int j0 = -1, j1 = -1;
    const float* a = des_tpl + (size_t)i * D;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < ncand) {
        const int j = t.j[k];
        top2_insert_exact(d0, j0, d1, j1, exact_dist_any(a, base + (size_t)j * D, D), j);
      }
    }
    out_idx[o] = j0;
    out_idx[o + 1] = j1;
    out_dist[o] = d0;
    out_dist[o + 1] = d1;
  }
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
                                                                         unsigned long long* __restrict__ fb_keys) {
  __shared__ __attribute__((aligned(16))) float sa[kFbBatch][kDP];
  __shared__ float sd[kFbThreads / 64][kFbBatch][2];
  __shared__ int sj[kFbThreads / 64][kFbBatch][2];
  const int f = blockIdx.x;
  const int cnt = fb_cnt[f];
  if (cnt <= (int)blockIdx.z * kFbBatch) return;  // the whole workgroup: no batch for it
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q_begin = q_off[f], n_q = q_off[f + 1] - q_begin;
  const int j_lo = (int)((long long)n_q * blockIdx.y / kFbSplit);
  const int j_hi = (int)((long long)n_q * (blockIdx.y + 1) / kFbSplit);
  const bool v4 = (D & 3) == 0 && (reinterpret_cast<uintptr_t>(des_q) & 15) == 0;
  for (int k0 = blockIdx.z * kFbBatch; k0 < cnt; k0 += kFbLanes * kFbBatch) {
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

// The listed rows' merged keys -> out_idx / out_dist (no key: index -1, FLT_MAX).
__global__ __launch_bounds__(256) void knn2_l2f32_fallback_out_kernel(int n_tpl, const int32_t* __restrict__ fb,
                                                                      const int32_t* __restrict__ fb_cnt,
                                                                      const unsigned long long* __restrict__ fb_keys,
                                                                      int32_t* __restrict__ out_idx,
                                                                      float* __restrict__ out_dist) {
  const int f = blockIdx.x;
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

int launch_knn_f32(kcmc_ctx* ctx, const float* des_tpl, int n_tpl, int D, const float* des_q, const int32_t* q_off,
                   int n_frames, int max_nq, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  // workspace: per-frame fallback counters and lists (room for every template row), K,
  // the tiles' max |b|^2, then the tile images (tpf = ceil(max_nq / 32) per frame; the
  // CSR total is a device value)
  const size_t rows = (size_t)n_frames * n_tpl;
  const int tpf = ceil_div(max(max_nq, 0), kTile);
  const size_t cnt_bytes = ((size_t)n_frames * sizeof(int32_t) + 255) & ~(size_t)255;
  const size_t fb_bytes = (rows * sizeof(int32_t) + 255) & ~(size_t)255;
  const size_t norm_bytes = (256 + (size_t)n_frames * tpf * sizeof(float) + 255) & ~(size_t)255;
  const size_t img_bytes = (size_t)n_frames * tpf * kImgBytes;
  const size_t key_bytes = rows * 2 * sizeof(unsigned long long);  // the fallback's merged top-2 keys
  void* ws = nullptr;
  KCMC_TRY(workspace_alloc(ctx, &ws, cnt_bytes + fb_bytes + norm_bytes + img_bytes + key_bytes, s));
  char* w = static_cast<char*>(ws);
  int32_t* fb_cnt = reinterpret_cast<int32_t*>(w);
  int32_t* fb = reinterpret_cast<int32_t*>(w + cnt_bytes);
  unsigned* Kbits = reinterpret_cast<unsigned*>(w + cnt_bytes + fb_bytes);
  float* tile_max = reinterpret_cast<float*>(w + cnt_bytes + fb_bytes + 256);
  uint8_t* img = reinterpret_cast<uint8_t*>(w + cnt_bytes + fb_bytes + norm_bytes);
  unsigned long long* fb_keys = reinterpret_cast<unsigned long long*>(w + cnt_bytes + fb_bytes + norm_bytes + img_bytes);
  KCMC_TRY(hip_check(hipMemsetAsync(fb_cnt, 0, (size_t)n_frames * sizeof(int32_t), s), "hipMemsetAsync"));
  KCMC_TRY(hip_check(hipMemsetAsync(Kbits, 0, sizeof(unsigned), s), "hipMemsetAsync"));
  hipLaunchKernelGGL(tpl_norm_max_kernel, dim3(ceil_div(n_tpl, 8)), dim3(256), 0, s, des_tpl, n_tpl, D, Kbits);
  KCMC_TRY(launch_check("tpl_norm_max_kernel"));
  if (tpf > 0) {
    hipLaunchKernelGGL(split_tiles_kernel, dim3(tpf, n_frames), dim3(256), 0, s, des_q, D, q_off, tpf, Kbits, img,
                       tile_max);
    KCMC_TRY(launch_check("split_tiles_kernel"));
  }
  hipLaunchKernelGGL(knn2_l2f32_kernel, dim3(ceil_div(n_tpl, kTplPerWG), n_frames), dim3(kThreads), 0, s, des_tpl,
                     n_tpl, D, des_q, q_off, img, tpf, Kbits, tile_max, out_idx, out_dist, fb, fb_cnt);
  KCMC_TRY(launch_check("knn2_l2f32_kernel"));
  KCMC_TRY(hip_check(hipMemsetAsync(fb_keys, 0xff, key_bytes, s), "hipMemsetAsync"));
  hipLaunchKernelGGL(knn2_l2f32_fallback_kernel, dim3(n_frames, kFbSplit, kFbLanes), dim3(kFbThreads), 0, s, des_tpl, n_tpl, D,
                     des_q, q_off, fb, fb_cnt, fb_keys);
  KCMC_TRY(launch_check("knn2_l2f32_fallback_kernel"));
  hipLaunchKernelGGL(knn2_l2f32_fallback_out_kernel, dim3(n_frames), dim3(256), 0, s, n_tpl, fb, fb_cnt, fb_keys,
                     out_idx, out_dist);
  KCMC_TRY(launch_check("knn2_l2f32_fallback_out_kernel"));
  return workspace_free(ctx, ws, s);
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_knn2_l2f32(kcmc_ctx* ctx, const float* des_tpl, int n_tpl, int D, const float* des_q,
                               const int32_t* q_off, int n_frames, int max_nq, int32_t* out_idx, float* out_dist,
                               kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_knn2_l2f32: ctx is NULL");
  KCMC_TRY(check_f32_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  return launch_knn_f32(ctx, des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist,
                        (hipStream_t)stream);
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
