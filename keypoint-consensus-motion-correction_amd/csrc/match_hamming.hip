// K1h (opt-in, not the reference's matcher): batched k=2 Hamming matching of binary
// descriptors, cv2.BFMatcher(cv2.NORM_HAMMING).knnMatch(des_template, des_query, k=2).
//
// The reference matches with cv2.BFMatcher(crossCheck=False), i.e. NORM_L2 on the uint8
// descriptor bytes (VA:194-195, match.hip); for binary ORB / BRIEF / AKAZE-MLDB
// descriptors OpenCV's documented norm is NORM_HAMMING, which this kernel provides as an
// extension (stages.match_frames(..., norm="hamming")).  Parity: the oracle's
// kcmc_oracle_knn2_hamming (popcount of the XOR, top-2 by OpenCV's K-insertion: strict
// comparison, so the lower frame index wins ties; the distance is the bit count as a
// float).
//
// knn2_hamming_kernel -- persistent and template-stationary like knn2_l2u8_kernel: each
//   lane owns one template row (its descriptor words in registers), a workgroup of 4
//   waves covers 256 template rows and walks frames g, g + G, ...; the frame's rows are
//   staged in LDS in 256-row chunks (double-buffered, one barrier per chunk, rows padded
//   to 16 / 64 bytes with zeros on both sides so the padding XORs to 0) and read as
//   wave-uniform broadcasts.  Per frame row: DW x (v_xor + v_bcnt_u32 accumulate), then
//   the key (bits << 21 | row) and the top-2 update (v_med3_u32, v_min_u32).
#include <cfloat>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;  // 4 waves, one template row per lane
constexpr int kQChunk = 256;   // frame rows per LDS chunk (one row per thread when staging)
constexpr int kIdxBits = 21;   // frame rows < 2^21; the bit count (<= 512) sits above them
constexpr uint32_t kNoKey = 0xffffffffu;

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// 4 descriptor bytes at column col, zero past D
__device__ __forceinline__ uint32_t load4(const uint8_t* row, int col, int D) {
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) w |= (col + b < D ? (uint32_t)row[col + b] : 0u) << (8 * b);
  return w;
}

__device__ __forceinline__ uint4 load16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);  // global_load_dwordx4 (unaligned access is allowed for global memory)
  return v;
}

// bytes of word w (0..3) of 16-byte piece k inside the descriptor
__device__ __forceinline__ uint32_t byte_mask(int D, int k, int w) {
  const int n = D - 16 * k - 4 * w;
  return n >= 4 ? ~0u : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
}

template <int DP>
__global__ __launch_bounds__(kThreads) void knn2_hamming_kernel(const uint8_t* __restrict__ des_tpl, int n_tpl, int D,
                                                                const uint8_t* __restrict__ des_q,
                                                                const int32_t* __restrict__ q_off, int n_frames,
                                                                int n_tg, int32_t* __restrict__ out_idx,
                                                                float* __restrict__ out_dist) {
  constexpr int DW = DP / 4;   // words per padded row
  constexpr int NP = DP / 16;  // 16-byte pieces per padded row
  __shared__ __attribute__((aligned(16))) uint32_t qbuf[2][kQChunk * DW];

  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int tg = id % n_tg, g = id / n_tg, G = gridDim.x / n_tg;
  const int tid = threadIdx.x;
  const int i = tg * kThreads + tid;  // this lane's template row
  const int last_global = q_off[n_frames] - 1;

  uint32_t tw[DW];
#pragma unroll
  for (int k = 0; k < DW; ++k) tw[k] = i < n_tpl ? load4(des_tpl + (size_t)i * D, 4 * k, D) : 0u;

  // staging: thread tid loads frame row q0 + tid as NP 16-byte pieces (the last one may
  // run into the next row; masked when landing); des_q's very last row is read bytewise
  uint4 pf[NP];
  auto issue = [&](int qb, int nq, int q0) {
    const int r = qb + q0 + min(tid, nq - q0 - 1);
    const uint8_t* row = des_q + (size_t)r * D;
    const int np = (D + 15) >> 4;
#pragma unroll
    for (int k = 0; k < NP; ++k) pf[k] = load16(row + 16 * min(k, np - 1));
    if (r == last_global && (D & 15) != 0) {  // one lane in the grid: no read past des_q
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      for (int cc = 0; cc < 16; ++cc)
        if (16 * (np - 1) + cc < D) w[cc >> 2] |= (uint32_t)row[16 * (np - 1) + cc] << (8 * (cc & 3));
#pragma unroll
      for (int k = 0; k < NP; ++k)
        if (k == np - 1) pf[k] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  };
  auto next_frame = [&](int f) {
    for (f += G; f < n_frames && q_off[f + 1] == q_off[f]; f += G) {
    }
    return f;
  };
  {
    const int f1 = (g < n_frames && q_off[g + 1] > q_off[g]) ? g : next_frame(g);
    if (f1 < n_frames) issue(q_off[f1], q_off[f1 + 1] - q_off[f1], 0);
  }
  int buf = 0;
  for (int f = g; f < n_frames; f += G) {
    const int q_begin = q_off[f];
    const int n_q = q_off[f + 1] - q_begin;
    const int nf = next_frame(f);
    const int nqb = nf < n_frames ? q_off[nf] : 0;
    const int nnq = nf < n_frames ? q_off[nf + 1] - nqb : 0;
    uint32_t b1 = kNoKey, b2 = kNoKey;
    for (int q0 = 0; q0 < n_q; q0 += kQChunk, buf ^= 1) {
      const int cnt = min(kQChunk, n_q - q0);
      if (tid < cnt) {
        uint4* dst = reinterpret_cast<uint4*>(&qbuf[buf][tid * DW]);
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          uint4 v = pf[k];
          v.x &= byte_mask(D, k, 0);
          v.y &= byte_mask(D, k, 1);
          v.z &= byte_mask(D, k, 2);
          v.w &= byte_mask(D, k, 3);
          dst[k] = v;
        }
      }
      __syncthreads();
      if (q0 + kQChunk < n_q)
        issue(q_begin, n_q, q0 + kQChunk);
      else if (nf < n_frames)
        issue(nqb, nnq, 0);
      const uint32_t* qb = qbuf[buf];
      for (int j = 0; j < cnt; ++j) {
        const uint32_t* row = qb + j * DW;  // wave-uniform: LDS broadcast reads
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < DW; ++k) bits += __popc(tw[k] ^ row[k]);  // v_xor + v_bcnt_u32 (accumulating)
        const uint32_t key = (bits << kIdxBits) | (uint32_t)(q0 + j);
        b2 = med3_u32(b1, b2, key);
        b1 = min(b1, key);
      }
    }
    if (i < n_tpl) {
      const size_t o = ((size_t)f * n_tpl + i) * 2;
      const uint32_t ks[2] = {b1, b2};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        out_idx[o + k] = ks[k] == kNoKey ? -1 : (int32_t)(ks[k] & ((1u << kIdxBits) - 1u));
        out_dist[o + k] = ks[k] == kNoKey ? FLT_MAX : (float)(ks[k] >> kIdxBits);
      }
    }
  }
}

int check_hamming_args(const void* des_tpl, int n_tpl, int D, const void* des_q, const void* q_off, int n_frames,
                       int max_nq, const void* o1, const void* o2) {
  if (n_tpl < 0 || n_frames < 0 || max_nq < 0) return fail(KCMC_EINVAL, "match_hamming: negative size");
  if (D < 1 || D > 64)
    return fail(KCMC_EUNSUPPORTED, "match_hamming: descriptor length D must be in [1, 64] (got " + std::to_string(D) + ")");
  if (max_nq >= (1 << kIdxBits)) return fail(KCMC_EUNSUPPORTED, "match_hamming: at most 2^21 - 1 rows per frame");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "match_hamming: at most 65535 frames per call");
  if (n_frames > 0 && n_tpl > 0 && (!des_tpl || !q_off || !o1 || !o2 || (max_nq > 0 && !des_q)))
    return fail(KCMC_EINVAL, "match_hamming: NULL pointer");
  return KCMC_OK;
}

int launch_knn_hamming(const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q, const int32_t* q_off,
                       int n_frames, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  const int cus = device_cus();
  const int n_tg = ceil_div(n_tpl, kThreads);
  // workgroups per CU: LDS-bound (2 x 256 rows x 32 / 64 B per workgroup)
  const int G = std::max(1, std::min(n_frames, (D <= 32 ? 8 : 4) * cus / n_tg));
  if (D <= 32)
    hipLaunchKernelGGL(knn2_hamming_kernel<32>, dim3(n_tg * G), dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off,
                       n_frames, n_tg, out_idx, out_dist);
  else
    hipLaunchKernelGGL(knn2_hamming_kernel<64>, dim3(n_tg * G), dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off,
                       n_frames, n_tg, out_idx, out_dist);
  return launch_check("knn2_hamming_kernel");
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_knn2_hamming(kcmc_ctx* ctx, const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q,
                                 const int32_t* q_off, int n_frames, int max_nq, int32_t* out_idx, float* out_dist,
                                 kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_knn2_hamming: ctx is NULL");
  KCMC_TRY(check_hamming_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  return launch_knn_hamming(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, (hipStream_t)stream);
}

extern "C" int kcmc_match_frames_hamming(kcmc_ctx* ctx, const uint8_t* des_tpl, const double* kp_tpl, int n_tpl, int D,
                                         const uint8_t* des_q, const double* kp_q, const int32_t* q_off, int n_frames,
                                         int max_nq, double ratio, double d_lo, double d_hi, int32_t* out_idx,
                                         float* out_dist, double* out_kp_ordered, uint32_t* out_keep_bits,
                                         int32_t* out_counts, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_match_frames_hamming: ctx is NULL");
  KCMC_TRY(check_hamming_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  if (n_frames > 0 && n_tpl > 0 && (!kp_tpl || !out_kp_ordered || !out_keep_bits || !out_counts || (max_nq > 0 && !kp_q)))
    return fail(KCMC_EINVAL, "kcmc_match_frames_hamming: NULL pointer");
  if (n_tpl > 8192) return fail(KCMC_EUNSUPPORTED, "kcmc_match_frames_hamming: n_tpl > 8192");
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  hipStream_t s = (hipStream_t)stream;
  KCMC_TRY(launch_knn_hamming(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s));
  return launch_match_filter(out_idx, out_dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio, d_lo, d_hi,
                             out_kp_ordered, out_keep_bits, out_counts, s);
}
