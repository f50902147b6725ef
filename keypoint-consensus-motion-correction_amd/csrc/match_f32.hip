// K1f: batched k=2 L2 matching of float32 descriptors (SIFT-style, BASELINE config 5).
//
// The reference matches uint8 AKAZE/BRISK descriptors (VA:194-195, match.hip); config 5
// asks for float descriptors, where the distance is a genuine dense fp32 contraction.
// Distance definition (OpenCV's batchDistL2_32f accumulates in a
// build-dependent SIMD order, so parity with it is unpinned): the near-exact
//   S = sum_k ((double)a_k - (double)b_k)^2 (sequential, fp64), dist = sqrtf((float)S),
// top-2 by (dist, frame index) like OpenCV's K-insertion.
//
// split_rows_kernel -- once per call: every frame row as bf16 hi | lo (v = hi + lo + e,
//   |e| <= 2^-18 |v|; hi = RNE(v), v - hi exact, lo = RNE(v - hi)) and its fp32 squared
//   norm, so that the template blocks of a frame share one conversion.
//
// knn2_l2f32_kernel -- one workgroup = 128 template rows x one frame (4 waves x one block
//   of 32 rows; 3 waves per SIMD, several workgroups per CU so that one workgroup's
//   barriers overlap another's matrix work).  Phase 1 on the bf16 matrix cores:
//   d~ = |a|^2 + |b|^2 - 2 a.b with a.b ~ hi.hi + hi.lo + lo.hi by
//   v_mfma_f32_32x32x16_bf16 (3 MFMAs per k-step of 16: 5.3x fewer cycles than
//   v_mfma_f32_32x32x2_f32 for the same contraction).  B = the 32 template rows, split in
//   registers; A = 32 frame rows per chunk, copied from the split rows into LDS (the next
//   chunk's loads in flight during the current chunk's MFMAs).  Each lane keeps its
//   template row's chunk top-4 on 32-bit keys (d~'s float bits with the low 6 mantissa
//   bits replaced by the chunk-local row, 4 VALU per distance) and folds it into a running
//   approximate top-4.  The error of a listed value is bounded by
//     eps = (6 (D + 4) 2^-24 + 2^-15) (|a| + max|b|)^2
//   (derivation at its use below).
//   A frame row can be among the exact top-2 only if d~ <= d~(2) + 2 eps, so when the
//   approximate 4th value exceeds that bound the exact top-2 lies within the top-3
//   candidates: phase 2 re-evaluates them with the exact fp64 definition and orders
//   them by (dist, index).  Rows that cannot be certified (near-ties of 4+ frame
//   descriptors) are appended to a list that knn2_l2f32_fallback_kernel finishes by
//   exact brute force, one wave per row.
#include <cfloat>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 256;
constexpr int kBlocks = 1;                         // 32-row template blocks per wave (2: 1 wave per SIMD)
constexpr int kTplPerWG = (kThreads / 64) * kBlocks * 32;  // 128
constexpr int kDP = 128;                           // padded descriptor length
constexpr int kKSteps = kDP / 16;                  // k-steps of v_mfma_f32_32x32x16_bf16
constexpr int kQChunk = 32;                        // frame rows per LDS chunk (one MFMA tile; local index < 64)
constexpr int kRowB = kDP + 8;                     // padded LDS row (bf16 elements, 272 B)
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

// Frame rows split once for every template block: row q -> bf16 hi[128] | lo[128] (zero
// past D) and its fp32 squared norm.  32 lanes per row, 4 floats each.
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ des_q, int D,
                                                         const int32_t* __restrict__ q_off, int n_frames,
                                                         uint2* __restrict__ qsplit, float* __restrict__ qnorm,
                                                         long long qrows) {
  const int f = blockIdx.y;
  const int q = q_off[f] + blockIdx.x * 8 + (threadIdx.x >> 5);
  if (q >= q_off[f + 1] || q >= qrows) return;  // whole 32-lane groups exit together
  const int col = (threadIdx.x & 31) * 4;
  const float* src = des_q + (size_t)q * D;
  float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((D & 3) == 0 && (reinterpret_cast<uintptr_t>(des_q) & 15) == 0) {
    if (col < D) w = *reinterpret_cast<const float4*>(src + col);
  } else {
    w.x = col < D ? src[col] : 0.f;
    w.y = col + 1 < D ? src[col + 1] : 0.f;
    w.z = col + 2 < D ? src[col + 2] : 0.f;
    w.w = col + 3 < D ? src[col + 3] : 0.f;
  }
  float ss = fmaf(w.w, w.w, fmaf(w.z, w.z, fmaf(w.y, w.y, w.x * w.x)));
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
  if ((threadIdx.x & 31) == 0) qnorm[q] = ss;
  __bf16 hv[4], lv[4];
  split_bf16(w.x, hv[0], lv[0]);
  split_bf16(w.y, hv[1], lv[1]);
  split_bf16(w.z, hv[2], lv[2]);
  split_bf16(w.w, hv[3], lv[3]);
  qsplit[(size_t)q * 64 + (threadIdx.x & 31)] = *reinterpret_cast<const uint2*>(hv);
  qsplit[(size_t)q * 64 + 32 + (threadIdx.x & 31)] = *reinterpret_cast<const uint2*>(lv);
}

// Loads of one chunk of split frame rows (32 x 16 B per row; 4 pieces per thread at 512
// threads, in named registers: an indexed array here was placed in scratch memory),
// addresses clamped to the frame's last row (and to the split buffer, should max_nq
// undercount).
static_assert(kQChunk * 32 / kThreads == 4, "issue_chunk loads four 16-byte pieces per thread");
__device__ __forceinline__ uint4 chunk_piece(const uint4* __restrict__ qs, int q0n, int e, int last, int first) {
  return qs[(size_t)(q0n + max(min(e >> 5, last), first)) * 32 + (e & 31)];
}
__device__ __forceinline__ void issue_chunk(const uint4* __restrict__ qs, const float* __restrict__ qnorm,
                                            long long qrows, int q_begin, int n_q, int q0n, int tid, uint4& p0,
                                            uint4& p1, uint4& p2, uint4& p3, float& pn) {
  const int last = (int)min((long long)(n_q - 1 - q0n), qrows - 1 - q_begin - q0n);
  const int first = -q_begin - q0n;
  p0 = chunk_piece(qs, q0n, tid, last, first);
  p1 = chunk_piece(qs, q0n, tid + kThreads, last, first);
  p2 = chunk_piece(qs, q0n, tid + 2 * kThreads, last, first);
  p3 = chunk_piece(qs, q0n, tid + 3 * kThreads, last, first);
  if (tid < kQChunk) pn = qnorm[q_begin + q0n + max(min(tid, last), first)];
}

__device__ __forceinline__ void land_piece(__bf16* qhi, __bf16* qlo, int e, const uint4& v) {
  const int r = e >> 5, part = e & 31;
  __bf16* dstp = (part < 16 ? qhi : qlo) + r * kRowB + 8 * (part & 15);
  *reinterpret_cast<uint4*>(dstp) = v;
}

__global__ __launch_bounds__(kThreads) void knn2_l2f32_kernel(
    const float* __restrict__ des_tpl, int n_tpl, int D, const float* __restrict__ des_q,
    const int32_t* __restrict__ q_off, const uint2* __restrict__ qsplit, const float* __restrict__ qnorm,
    long long qrows, int32_t* __restrict__ out_idx, float* __restrict__ out_dist, int32_t* __restrict__ fallback,
    int32_t* __restrict__ n_fallback) {
  __shared__ __attribute__((aligned(16))) __bf16 qhi[kQChunk * kRowB];
  __shared__ __attribute__((aligned(16))) __bf16 qlo[kQChunk * kRowB];
  __shared__ float qn[kQChunk];
  __shared__ unsigned s_maxqn;  // max |b|^2 over the frame (float bits; positive floats order as ints)

  // XCD-aware order: the workgroups of one frame get consecutive ids of one XCD's run
  // (dispatch is round-robin over the 8 XCDs), so the frame's descriptors stay in that
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
  if (tid == 0) s_maxqn = 0u;

  // ---- template fragments (B operand, bf16 hi/lo split) kept in registers: lane (c, h)
  // holds row i's elements k = 16 s + 8 h + j of k-step s; and the row's squared norm
  bf16x8 bhi[kBlocks][kKSteps], blo[kBlocks][kKSteps];
  float tn[kBlocks];
  int tpl_row[kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const int i = tb * kTplPerWG + (wave * kBlocks + b) * 32 + c;
    tpl_row[b] = i;
    float na = 0.f;
#pragma unroll
    for (int st = 0; st < kKSteps; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * st + 8 * h + j;
        const float v = (i < n_tpl && k < D) ? des_tpl[(size_t)i * D + k] : 0.f;
        __bf16 hv, lv;
        split_bf16(v, hv, lv);
        bhi[b][st][j] = hv;
        blo[b][st][j] = lv;
        na = fmaf(v, v, na);
      }
    tn[b] = na + __shfl_xor(na, 32);
  }

  Top4 best[kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
#pragma unroll
    for (int k = 0; k < 4; ++k) best[b].v[k] = INFINITY;
#pragma unroll
    for (int k = 0; k < 3; ++k) best[b].j[k] = -1;
  }

  const float* base = des_q + (size_t)q_begin * D;
  // staging: the frame's rows were split once by split_rows_kernel (bf16 hi | lo, 512 B
  // per row, and the fp32 squared norm), so a chunk is a plain copy of 64 x 512 B; the
  // next chunk's loads are issued before the current chunk's MFMA tiles so that their
  // latency is hidden behind them.  Addresses are clamped to the frame's last row (the
  // tile outputs of rows >= cnt are never listed).
  const uint4* qs = reinterpret_cast<const uint4*>(qsplit) + (size_t)q_begin * 32;
  uint4 p0, p1, p2, p3;
  float pn = 0.f;
  if (n_q > 0) issue_chunk(qs, qnorm, qrows, q_begin, n_q, 0, tid, p0, p1, p2, p3, pn);
  for (int q0 = 0; q0 < n_q; q0 += kQChunk) {
    const int cnt = min(kQChunk, n_q - q0);
    __syncthreads();  // previous chunk consumed
    land_piece(qhi, qlo, tid, p0);
    land_piece(qhi, qlo, tid + kThreads, p1);
    land_piece(qhi, qlo, tid + 2 * kThreads, p2);
    land_piece(qhi, qlo, tid + 3 * kThreads, p3);
    if (tid < kQChunk) {
      qn[tid] = pn;
      if (tid < cnt) atomicMax(&s_maxqn, __float_as_uint(pn));
    }
    __syncthreads();
    if (q0 + kQChunk < n_q) issue_chunk(qs, qnorm, qrows, q_begin, n_q, q0 + kQChunk, tid, p0, p1, p2, p3, pn);
    // ---- 32-row tiles: a.b ~ hi.hi + hi.lo + lo.hi on the bf16 matrix cores (fp32
    // accumulation); the chunk's top-4 per lane on 32-bit keys (d~ with the low 6
    // mantissa bits replaced by the chunk-local row)
    uint32_t ck[kBlocks][4];
#pragma unroll
    for (int b = 0; b < kBlocks; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k) ck[b][k] = kNoKey;
    for (int t0 = 0; t0 < cnt; t0 += 32) {
      v16f acc[kBlocks];
#pragma unroll
      for (int b = 0; b < kBlocks; ++b) acc[b] = v16f{0.f};
      const __bf16* ah = &qhi[(t0 + c) * kRowB + 8 * h];
      const __bf16* al = &qlo[(t0 + c) * kRowB + 8 * h];
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
      // lane's 16 accumulators: chunk rows t0 + (r & 3) + 8 (r >> 2) + 4h of column c
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool ok = row < cnt;
        const float qv = qn[row];
#pragma unroll
        for (int b = 0; b < kBlocks; ++b) {
          const float x = fmaf(-2.f, acc[b][r], tn[b] + qv);
          // negative d~ -> +0 (signed max on the bits); NaN sorts after every finite key
          const uint32_t xb = (uint32_t)max(__float_as_int(x), 0);
          top4_key(ck[b], ok ? ((xb & ~63u) | (uint32_t)row) : kNoKey);
        }
      }
    }
    // ---- fold the chunk's top-4 into the running top-4 (the chunk's 4th key bounds
    // every row of the chunk it did not report, and so does the running 4th value)
#pragma unroll
    for (int b = 0; b < kBlocks; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (ck[b][k] != kNoKey) top4_insert(best[b], __uint_as_float(ck[b][k] & ~63u), q0 + (int)(ck[b][k] & 63u));
  }
  __syncthreads();
  const float maxb = sqrtf(__uint_as_float(s_maxqn));

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
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const int i = tpl_row[b];
    if (i >= n_tpl) continue;
    const Top4& t = best[b];
    const float ra = sqrtf(fmaxf(tn[b], 0.f));
    // |d~ - d| <= eps for every listed value (units U = (|a| + max|b|)^2): norms 2 D u,
    // 2 a.b through bf16x3 <= (3D 2u + 3 2^-18) U / 2 (split residual + fp32 accumulation
    // of 3D exact bf16 products, rounding or truncating), two final roundings, and the
    // key truncation 2^-17; bounded with margin by (6 (D + 4) u + 2^-15) U, u = 2^-24.
    const float U = (ra + maxb) * (ra + maxb);
    const float eps = (6.f * (float)(D + 4) * 5.9604645e-8f + 3.0517578e-5f) * U * 1.01f + 1e-30f;
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
    if (ncand < 0) {
      const int slot = atomicAdd(n_fallback, 1);
      fallback[slot] = (int32_t)((size_t)f * n_tpl + i);
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

// Exact brute force for the rows phase 1 could not certify: one wave per row, lanes
// stride over the frame's rows, then a wave-wide lexicographic top-2 merge.  Every wave
// exits once the list is exhausted.
__global__ __launch_bounds__(256) void knn2_l2f32_fallback_kernel(const float* __restrict__ des_tpl, int n_tpl, int D,
                                                                  const float* __restrict__ des_q,
                                                                  const int32_t* __restrict__ q_off,
                                                                  const int32_t* __restrict__ fallback,
                                                                  const int32_t* __restrict__ n_fallback,
                                                                  int32_t* __restrict__ out_idx,
                                                                  float* __restrict__ out_dist) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  const int n = *n_fallback;
  for (int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w < n; w += nw) {
    const int fi = fallback[w];
    const int f = fi / n_tpl, i = fi - f * n_tpl;
    const int q_begin = q_off[f], n_q = q_off[f + 1] - q_begin;
    const float* a = des_tpl + (size_t)i * D;
    float d0 = FLT_MAX, d1 = FLT_MAX;
    int j0 = -1, j1 = -1;
    for (int j = lane; j < n_q; j += 64)
      top2_insert_exact(d0, j0, d1, j1, exact_dist_any(a, des_q + (size_t)(q_begin + j) * D, D), j);
    for (int off = 32; off > 0; off >>= 1) {
      const float e0 = __shfl_xor(d0, off), e1 = __shfl_xor(d1, off);
      const int k0 = __shfl_xor(j0, off), k1 = __shfl_xor(j1, off);
      if (k0 >= 0) top2_insert_exact(d0, j0, d1, j1, e0, k0);
      if (k1 >= 0) top2_insert_exact(d0, j0, d1, j1, e1, k1);
    }
    if (lane == 0) {
      const size_t o = (size_t)fi * 2;
      out_idx[o] = j0;
      out_idx[o + 1] = j1;
      out_dist[o] = d0;
      out_dist[o + 1] = d1;
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
  // workspace: fallback counter + list, then the split frame rows (512 B each) and their
  // norms, sized for n_frames * max_nq rows (the CSR total is a device value)
  const size_t rows = (size_t)n_frames * n_tpl;
  const size_t qrows = (size_t)n_frames * (size_t)max(max_nq, 0);
  const size_t fb_bytes = ((rows + 1) * sizeof(int32_t) + 255) & ~(size_t)255;
  void* ws = nullptr;
  KCMC_TRY(workspace_alloc(ctx, &ws, fb_bytes + qrows * 512 + qrows * sizeof(float), s));
  int32_t* n_fb = static_cast<int32_t*>(ws);
  int32_t* fb = n_fb + 1;
  uint2* qsplit = reinterpret_cast<uint2*>(static_cast<char*>(ws) + fb_bytes);
  float* qnorm = reinterpret_cast<float*>(static_cast<char*>(ws) + fb_bytes + qrows * 512);
  KCMC_TRY(hip_check(hipMemsetAsync(n_fb, 0, sizeof(int32_t), s), "hipMemsetAsync"));
  if (max_nq > 0) {
    hipLaunchKernelGGL(split_rows_kernel, dim3(ceil_div(max_nq, 8), n_frames), dim3(256), 0, s, des_q, D, q_off,
                       n_frames, qsplit, qnorm, (long long)qrows);
    KCMC_TRY(launch_check("split_rows_kernel"));
  }
  hipLaunchKernelGGL(knn2_l2f32_kernel, dim3(ceil_div(n_tpl, kTplPerWG), n_frames), dim3(kThreads), 0, s, des_tpl,
                     n_tpl, D, des_q, q_off, qsplit, qnorm, (long long)qrows, out_idx, out_dist, fb, n_fb);
  KCMC_TRY(launch_check("knn2_l2f32_kernel"));
  hipLaunchKernelGGL(knn2_l2f32_fallback_kernel, dim3(512), dim3(256), 0, s, des_tpl, n_tpl, D, des_q, q_off, fb, n_fb,
                     out_idx, out_dist);
  KCMC_TRY(launch_check("knn2_l2f32_fallback_kernel"));
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
