// K1f: batched k=2 L2 matching of float32 descriptors (SIFT-style, BASELINE config 5).
//
// The reference matches uint8 AKAZE/BRISK descriptors (VA:194-195, match.hip); config 5
// asks for float descriptors, where the distance is a genuine dense fp32 contraction.
// Distance definition (OpenCV's batchDistL2_32f accumulates in a
// build-dependent SIMD order, so parity with it is unpinned): the near-exact
//   S = sum_k ((double)a_k - (double)b_k)^2 (sequential, fp64), dist = sqrtf((float)S),
// top-2 by (dist, frame index) like OpenCV's K-insertion.
//
// knn2_l2f32_kernel -- one workgroup = 256 template rows x one frame (4 waves x 2 blocks
//   of 32 rows).  Phase 1 on the matrix cores: d~ = |a|^2 + |b|^2 - 2 a.b with
//   v_mfma_f32_32x32x2_f32 (B = 32 template rows held in registers, A = 32 frame rows
//   streamed from LDS in 64-row chunks); each lane keeps the approximate top-4 of its
//   template row.  The fp32 error of d~ is bounded by
//     eps = 2 (D + 4) 2^-24 (|a| + max|b|)^2
//   (norms and dot product each within gamma_D of exact, two more roundings, 2x slack).
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

constexpr int kThreads = 256;
constexpr int kBlocks = 2;                         // 32-row template blocks per wave
constexpr int kTplPerWG = (kThreads / 64) * kBlocks * 32;  // 256
constexpr int kDP = 128;                           // padded descriptor length (floats)
constexpr int kHalf = kDP / 2;                     // MFMA k-half: lane half h covers k in [64h, 64h+64)
constexpr int kQChunk = 64;                        // frame rows per LDS chunk
constexpr int kRow = kDP + 4;                      // padded LDS row (floats)

// The build's exact distance (identical operation order in the oracle).
__device__ __forceinline__ float exact_dist(const float* __restrict__ a, const float* __restrict__ b, int D) {
  double S = 0.0;
  for (int k = 0; k < D; ++k) {
    const double t = (double)a[k] - (double)b[k];
    S += t * t;
  }
  return sqrtf((float)S);
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

__global__ __launch_bounds__(kThreads) void knn2_l2f32_kernel(
    const float* __restrict__ des_tpl, int n_tpl, int D, const float* __restrict__ des_q,
    const int32_t* __restrict__ q_off, int32_t* __restrict__ out_idx, float* __restrict__ out_dist,
    int32_t* __restrict__ fallback, int32_t* __restrict__ n_fallback) {
  __shared__ __attribute__((aligned(16))) float qbuf[kQChunk * kRow];
  __shared__ float qn[kQChunk];
  __shared__ unsigned s_maxqn;  // max |b|^2 over the frame (float bits; positive floats order as ints)

  const int f = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31;  // MFMA column = template row within a block
  const int h = lane >> 5;  // k-half of the fragments / row group of the output
  const int q_begin = q_off[f];
  const int n_q = q_off[f + 1] - q_begin;
  if (tid == 0) s_maxqn = 0u;

  // ---- template fragments (B operand) kept in registers: lane (c, h) holds row i's
  // elements k = 64h + s, s = 0..63, and the row's squared norm (fp32)
  float bfrag[kBlocks][kHalf];
  float tn[kBlocks];
  int tpl_row[kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const int i = blockIdx.x * kTplPerWG + (wave * kBlocks + b) * 32 + c;
    tpl_row[b] = i;
    float na = 0.f;
#pragma unroll
    for (int s = 0; s < kHalf; ++s) {
      const int k = kHalf * h + s;
      const float v = (i < n_tpl && k < D) ? des_tpl[(size_t)i * D + k] : 0.f;
      bfrag[b][s] = v;
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
  const bool vec = (D & 3) == 0;
  for (int q0 = 0; q0 < n_q; q0 += kQChunk) {
    const int cnt = min(kQChunk, n_q - q0);
    __syncthreads();  // previous chunk consumed
    // ---- stage frame rows [q0, q0 + cnt) zero-padded to kDP floats
    for (int e = tid; e < kQChunk * (kDP / 4); e += kThreads) {
      const int r = e / (kDP / 4), col = (e % (kDP / 4)) * 4;
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < cnt && col < D) {
        const float* src = base + (size_t)(q0 + r) * D + col;
        if (vec) {
          w = *reinterpret_cast<const float4*>(src);
        } else {
          w.x = src[0];
          w.y = col + 1 < D ? src[1] : 0.f;
          w.z = col + 2 < D ? src[2] : 0.f;
          w.w = col + 3 < D ? src[3] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(&qbuf[r * kRow + col]) = w;
    }
    __syncthreads();
    if (tid < kQChunk) {
      float nb = 0.f;
      const float4* rw = reinterpret_cast<const float4*>(&qbuf[tid * kRow]);
#pragma unroll 8
      for (int d = 0; d < kDP / 4; ++d) {
        const float4 v = rw[d];
        nb = fmaf(v.x, v.x, nb);
        nb = fmaf(v.y, v.y, nb);
        nb = fmaf(v.z, v.z, nb);
        nb = fmaf(v.w, v.w, nb);
      }
      qn[tid] = nb;
      if (tid < cnt) atomicMax(&s_maxqn, __float_as_uint(nb));
    }
    __syncthreads();
    // ---- 32-row MFMA tiles
    for (int t0 = 0; t0 < cnt; t0 += 32) {
      v16f acc[kBlocks];
#pragma unroll
      for (int b = 0; b < kBlocks; ++b) acc[b] = v16f{0.f};
      const float* arow = &qbuf[(t0 + c) * kRow + kHalf * h];
#pragma unroll
      for (int s4 = 0; s4 < kHalf; s4 += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(arow + s4);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int b = 0; b < kBlocks; ++b)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bfrag[b][s4 + u], acc[b], 0, 0, 0);
      }
      // lane's 16 accumulators: frame rows t0 + (r & 3) + 8 (r >> 2) + 4h of column c
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool ok = row < cnt;
        const float qv = qn[row & (kQChunk - 1)];
#pragma unroll
        for (int b = 0; b < kBlocks; ++b) {
          const float x = ok ? fmaf(-2.f, acc[b][r], tn[b] + qv) : INFINITY;
          top4_insert(best[b], x, q0 + row);
        }
      }
    }
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
    const float eps = 2.f * (float)(D + 4) * 5.9604645e-8f * (ra + maxb) * (ra + maxb) * 1.01f + 1e-30f;
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
        top2_insert_exact(d0, j0, d1, j1, exact_dist(a, base + (size_t)j * D, D), j);
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
      top2_insert_exact(d0, j0, d1, j1, exact_dist(a, des_q + (size_t)(q_begin + j) * D, D), j);
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
                   int n_frames, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  void* ws = nullptr;
  const size_t rows = (size_t)n_frames * n_tpl;
  KCMC_TRY(workspace_alloc(ctx, &ws, (rows + 1) * sizeof(int32_t), s));
  int32_t* n_fb = static_cast<int32_t*>(ws);
  int32_t* fb = n_fb + 1;
  KCMC_TRY(hip_check(hipMemsetAsync(n_fb, 0, sizeof(int32_t), s), "hipMemsetAsync"));
  hipLaunchKernelGGL(knn2_l2f32_kernel, dim3(ceil_div(n_tpl, kTplPerWG), n_frames), dim3(kThreads), 0, s, des_tpl,
                     n_tpl, D, des_q, q_off, out_idx, out_dist, fb, n_fb);
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
  return launch_knn_f32(ctx, des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, (hipStream_t)stream);
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
  KCMC_TRY(launch_knn_f32(ctx, des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s));
  return launch_match_filter(out_idx, out_dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio, d_lo, d_hi,
                             out_kp_ordered, out_keep_bits, out_counts, s);
}
