// K1: batched k=2 L2 matching of uint8 descriptors + the per-frame match filters.
//
// Reference: VA:194-214 (cv2.BFMatcher(crossCheck=False).knnMatch(des_template,
// des_query, k=2), best-match reorder, ratio filter, median displacement filter).
//
// knn2_l2u8_kernel -- one workgroup = 256 template rows x one frame.
//   The distance is an exact integer contraction, so it runs on the int8 matrix
//   cores: with x = a - 128 and y = b - 128 (int8), SSD = |x|^2 + |y|^2 - 2 x.y and
//   x.y comes from v_mfma_i32_32x32x32_i8.  A operand = 32 frame descriptors (rows j),
//   B operand = 32 template descriptors (columns i), so each lane owns one template
//   column and 16 frame rows of the 32x32 tile and keeps a running top-2 in
//   registers.  The top-2 runs on packed keys (ssd << jb | j): for D <= 64 bytes
//   sqrtf is strictly increasing on the integer SSD range, so integer
//   keys order exactly like OpenCV's float distances, and the low bits make ties go
//   to the lower frame index like OpenCV's K-insertion.  4 VALU ops per distance
//   (key = tk + qk - g*2^(jb+1); min; med3).  Frame descriptors are staged through
//   LDS in 256-row chunks (converted to int8, zero-padded to DP, rows padded by 16 B
//   so the ds_read_b128 fragment reads are bank-conflict free).
//
// match_filter_kernel -- one workgroup per frame: VA:196-214 in float64 with the
//   reference's exact operation order (no FMA contraction; file built with
//   -ffp-contract=off), median by an LDS bitonic sort.
#include <cfloat>
#include <climits>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kBlocksPerWave = 2;                         // 32-row template blocks per wave
constexpr int kTplPerWG = (kThreads / 64) * kBlocksPerWave * 32;  // 256
constexpr int kQChunk = 256;                              // frame descriptors per LDS chunk

template <bool WIDE>
struct KeyT;
template <>
struct KeyT<false> {
  using T = uint32_t;
  static constexpr T kMax = 0xffffffffu;
};
template <>
struct KeyT<true> {
  using T = unsigned long long;
  static constexpr T kMax = ~0ull;
};

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b) { return a < b ? a : b; }

template <typename K>
__device__ __forceinline__ void top2_insert(K& b1, K& b2, K key) {
  // b1 <= b2 always; new b2 = median(b1, b2, key), new b1 = min(b1, key).
  K hi = b1 > key ? b1 : key;
  b2 = b2 < hi ? b2 : hi;
  b1 = b1 < key ? b1 : key;
}

// Signed-byte view of 4 consecutive descriptor bytes at column `col` (zero past D).
__device__ __forceinline__ uint32_t load4_signed(const uint8_t* row, int col, int D) {
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    uint32_t v = (col + b < D) ? (uint32_t)(row[col + b] ^ 0x80u) : 0u;
    w |= v << (8 * b);
  }
  return w;
}

template <int DP, bool WIDE>
__global__ __launch_bounds__(kThreads) void knn2_l2u8_kernel(
    const uint8_t* __restrict__ des_tpl, int n_tpl, int D, const uint8_t* __restrict__ des_q,
    const int32_t* __restrict__ q_off, int jb, int32_t* __restrict__ out_idx,
    float* __restrict__ out_dist) {
  using K = typename KeyT<WIDE>::T;
  constexpr int KSTEPS = DP / 32;
  constexpr int ROWB = DP + 16;  // padded LDS row stride (bytes)
  __shared__ __attribute__((aligned(16))) uint8_t qbuf[kQChunk * ROWB];
  __shared__ __attribute__((aligned(16))) K qkey[kQChunk];

  const int f = blockIdx.y;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c = lane & 31;   // MFMA column (template row within a block)
  const int h = lane >> 5;   // k-half of the fragment / row group of the output
  const int q_begin = q_off[f];
  const int n_q = q_off[f + 1] - q_begin;
  const K jmask = (K)((1ull << jb) - 1ull);

  // ---- template fragments (B operand) and their squared norms, kept in registers
  v4i bfrag[kBlocksPerWave][KSTEPS];
  K tk[kBlocksPerWave];
  int tpl_row[kBlocksPerWave];
#pragma unroll
  for (int b = 0; b < kBlocksPerWave; ++b) {
    const int i = blockIdx.x * kTplPerWG + (wave * kBlocksPerWave + b) * 32 + c;
    tpl_row[b] = i;
    int na = 0;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      if (i < n_tpl) {
        const uint8_t* row = des_tpl + (size_t)i * D;
#pragma unroll
        for (int d = 0; d < 4; ++d) w[d] = load4_signed(row, 32 * kk + 16 * h + 4 * d, D);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) na = __builtin_amdgcn_sdot4((int)w[d], (int)w[d], na, false);
      bfrag[b][kk] = v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    }
    na += __shfl_xor(na, 32);
    tk[b] = WIDE ? (K)na : ((K)na << jb);
  }

  K best1[kBlocksPerWave], best2[kBlocksPerWave];
#pragma unroll
  for (int b = 0; b < kBlocksPerWave; ++b) best1[b] = best2[b] = KeyT<WIDE>::kMax;

  for (int q0 = 0; q0 < n_q; q0 += kQChunk) {
    const int cnt = min(kQChunk, n_q - q0);
    const int rows = (cnt + 31) & ~31;
    __syncthreads();  // previous chunk fully consumed
    // ---- stage frame descriptors [q0, q0+cnt) as int8, zero-padded to DP columns
    const uint8_t* base = des_q + (size_t)(q_begin + q0) * D;
    for (int e = tid; e < rows * (DP / 4); e += kThreads) {
      const int r = e / (DP / 4);
      const int col = (e % (DP / 4)) * 4;
      uint32_t w = 0;
      if (r < cnt) {
        if ((D & 3) == 0) {
          w = (col < D) ? (*reinterpret_cast<const uint32_t*>(base + (size_t)r * D + col) ^ 0x80808080u) : 0u;
        } else {
          w = load4_signed(base + (size_t)r * D, col, D);
        }
      }
      *reinterpret_cast<uint32_t*>(&qbuf[r * ROWB + col]) = w;
    }
    __syncthreads();
    // ---- per-row key part: |y|^2 << jb | j
    for (int r = tid; r < rows; r += kThreads) {
      int nb = 0;
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(&qbuf[r * ROWB]);
#pragma unroll
      for (int d = 0; d < DP / 4; ++d) nb = __builtin_amdgcn_sdot4((int)rw[d], (int)rw[d], nb, false);
      const K j = (K)(q0 + r);
      qkey[r] = WIDE ? (((K)nb << 32) | j) : (((K)nb << jb) | j);
    }
    __syncthreads();
    // ---- MFMA tiles of 32 frame rows
    for (int t0 = 0; t0 < rows; t0 += 32) {
      v4i afrag[KSTEPS];
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk)
        afrag[kk] = *reinterpret_cast<const v4i*>(&qbuf[(t0 + c) * ROWB + 32 * kk + 16 * h]);
      // rows of this lane's 16 accumulators: t0 + (r&3) + 8*(r>>2) + 4*h
      K qk[16];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int s = 0; s < 4; ++s) qk[4 * g + s] = qkey[t0 + 8 * g + 4 * h + s];
      const bool partial = (t0 + 32 > cnt);
#pragma unroll
      for (int b = 0; b < kBlocksPerWave; ++b) {
        v16i acc = {0};
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk)
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag[kk], bfrag[b][kk], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          K key;
          if (WIDE) {
            // ssd = |x|^2 + |y|^2 - 2 x.y; key = ssd << 32 | j
            const long long ssd = (long long)tk[b] + (long long)(qk[r] >> 32) - 2ll * acc[r];
            key = ((K)ssd << 32) | (qk[r] & 0xffffffffull);
          } else {
            key = (K)(tk[b] + qk[r] - ((uint32_t)acc[r] << (jb + 1)));
          }
          if (partial) {
            const int row = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            key = (row < cnt) ? key : KeyT<WIDE>::kMax;
          }
          top2_insert(best1[b], best2[b], key);
        }
      }
    }
  }

  // ---- merge the two row halves (lanes l and l^32 own the same template column)
#pragma unroll
  for (int b = 0; b < kBlocksPerWave; ++b) {
    K o1, o2;
    if (WIDE) {
      o1 = (K)__shfl_xor((long long)best1[b], 32);
      o2 = (K)__shfl_xor((long long)best2[b], 32);
    } else {
      o1 = (K)__shfl_xor((int)best1[b], 32);
      o2 = (K)__shfl_xor((int)best2[b], 32);
    }
    const K m1 = best1[b] < o1 ? best1[b] : o1;
    const K hi = best1[b] < o1 ? o1 : best1[b];
    const K lo2 = best2[b] < o2 ? best2[b] : o2;
    const K m2 = hi < lo2 ? hi : lo2;
    const int i = tpl_row[b];
    if (h == 0 && i < n_tpl) {
      const size_t o = ((size_t)f * n_tpl + i) * 2;
      const K ms[2] = {m1, m2};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (ms[k] == KeyT<WIDE>::kMax) {
          out_idx[o + k] = -1;
          out_dist[o + k] = FLT_MAX;
        } else {
          const unsigned long long ssd = WIDE ? ((unsigned long long)ms[k] >> 32) : (unsigned long long)(ms[k] >> jb);
          out_idx[o + k] = (int32_t)(WIDE ? (ms[k] & 0xffffffffull) : (ms[k] & jmask));
          out_dist[o + k] = sqrtf((float)ssd);
        }
      }
    }
  }
}

// ------------------------------------------------------------ per-frame filters
constexpr int kFilterThreads = 256;

__global__ __launch_bounds__(kFilterThreads) void match_filter_kernel(
    const int32_t* __restrict__ idx, const float* __restrict__ dist, const double* __restrict__ kp_tpl,
    const double* __restrict__ kp_q, const int32_t* __restrict__ q_off, int n_tpl, double ratio,
    double d_lo, double d_hi, double* __restrict__ kp_ordered, uint32_t* __restrict__ keep_bits,
    int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) double sdisp[];  // [pow2 >= n_tpl]
  __shared__ int s_nratio;
  __shared__ int s_ndist;
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const int q_begin = q_off[f];
  const int words = (n_tpl + 31) >> 5;
  if (tid == 0) {
    s_nratio = 0;
    s_ndist = 0;
  }
  __syncthreads();

  // pass 1: reorder (VA:197-200), ratio filter (VA:202-203), displacement of survivors (VA:208)
  for (int i = tid; i < n_tpl; i += kFilterThreads) {
    const size_t o = ((size_t)f * n_tpl + i) * 2;
    const int j0 = idx[o];
    double qx = 0.0, qy = 0.0;
    if (j0 >= 0) {
      qx = kp_q[2 * (size_t)(q_begin + j0)];
      qy = kp_q[2 * (size_t)(q_begin + j0) + 1];
    }
    kp_ordered[((size_t)f * n_tpl + i) * 2] = qx;
    kp_ordered[((size_t)f * n_tpl + i) * 2 + 1] = qy;
    const bool ok = (double)dist[o] < ratio * (double)dist[o + 1];
    if (ok) {
      const double dx = kp_tpl[2 * i] - qx, dy = kp_tpl[2 * i + 1] - qy;
      const int p = atomicAdd(&s_nratio, 1);
      sdisp[p] = sqrt(dx * dx + dy * dy);
    }
  }
  __syncthreads();
  const int nr = s_nratio;
  int P = 1;
  while (P < nr) P <<= 1;
  for (int i = nr + tid; i < P; i += kFilterThreads) sdisp[i] = INFINITY;
  __syncthreads();
  // bitonic sort of the nr ratio-survivor displacements (np.median, VA:210)
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += kFilterThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double a = sdisp[i], b = sdisp[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            sdisp[i] = b;
            sdisp[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  double med = 0.0;
  if (nr > 0) med = (nr & 1) ? sdisp[nr >> 1] : (sdisp[(nr >> 1) - 1] + sdisp[nr >> 1]) / 2.0;
  const double lo = d_lo * med, hi = d_hi * med;

  // pass 2: keep = ratio survivor and lo <= d <= hi (VA:210); bitmask + counts
  const int lane = tid & 63;
  const int wave = tid >> 6;
  for (int base = 0; base < n_tpl; base += kFilterThreads) {
    const int i = base + tid;
    bool keep = false;
    if (i < n_tpl && nr > 0) {
      const size_t o = ((size_t)f * n_tpl + i) * 2;
      const bool ok = (double)dist[o] < ratio * (double)dist[o + 1];
      if (ok) {
        const double qx = kp_ordered[((size_t)f * n_tpl + i) * 2];
        const double qy = kp_ordered[((size_t)f * n_tpl + i) * 2 + 1];
        const double dx = kp_tpl[2 * i] - qx, dy = kp_tpl[2 * i + 1] - qy;
        const double d = sqrt(dx * dx + dy * dy);
        keep = (lo <= d) && (d <= hi);
      }
    }
    const unsigned long long m = __ballot(keep);
    const int w0 = (base + wave * 64) >> 5;
    if (lane == 0) {
      if (w0 < words) keep_bits[(size_t)f * words + w0] = (uint32_t)m;
      if (w0 + 1 < words) keep_bits[(size_t)f * words + w0 + 1] = (uint32_t)(m >> 32);
      if (m) atomicAdd(&s_ndist, __popcll(m));
    }
  }
  __syncthreads();
  if (tid == 0) {
    counts[4 * (size_t)f + 0] = n_tpl;  // len(kp_query) after the reorder at VA:200
    counts[4 * (size_t)f + 1] = n_tpl;  // len(matches)
    counts[4 * (size_t)f + 2] = nr;
    counts[4 * (size_t)f + 3] = s_ndist;
  }
}

int bits_for(long long v) {  // bits to represent 0..v
  int b = 1;
  while ((1ll << b) <= v) ++b;
  return b;
}

int launch_knn(const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q, const int32_t* q_off,
               int n_frames, int max_nq, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  const long long ssd_max = (long long)D * 255 * 255;
  const int jb = bits_for(max_nq > 0 ? max_nq - 1 : 0);
  const bool wide = (bits_for(ssd_max) + jb > 32) || ((((unsigned long long)ssd_max << jb) | ((1ull << jb) - 1)) >= 0xffffffffull);
  dim3 grid(ceil_div(n_tpl, kTplPerWG), n_frames);
  if (D <= 32) {
    if (wide)
      hipLaunchKernelGGL((knn2_l2u8_kernel<32, true>), grid, dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off, jb, out_idx, out_dist);
    else
      hipLaunchKernelGGL((knn2_l2u8_kernel<32, false>), grid, dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off, jb, out_idx, out_dist);
  } else {
    if (wide)
      hipLaunchKernelGGL((knn2_l2u8_kernel<64, true>), grid, dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off, jb, out_idx, out_dist);
    else
      hipLaunchKernelGGL((knn2_l2u8_kernel<64, false>), grid, dim3(kThreads), 0, s, des_tpl, n_tpl, D, des_q, q_off, jb, out_idx, out_dist);
  }
  return launch_check("knn2_l2u8_kernel");
}

int check_match_args(const void* des_tpl, int n_tpl, int D, const void* des_q, const void* q_off,
                     int n_frames, int max_nq, const void* o1, const void* o2) {
  if (n_tpl < 0 || n_frames < 0 || max_nq < 0) return fail(KCMC_EINVAL, "match: negative size");
  if (D < 1 || D > 64)
    return fail(KCMC_EUNSUPPORTED, "match: descriptor length D must be in [1, 64] (got " + std::to_string(D) + ")");
  if (max_nq > (1 << 30)) return fail(KCMC_EUNSUPPORTED, "match: max_nq too large");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "match: at most 65535 frames per call");
  if (n_frames > 0 && n_tpl > 0 && (!des_tpl || !q_off || !o1 || !o2 || (max_nq > 0 && !des_q)))
    return fail(KCMC_EINVAL, "match: NULL pointer");
  return KCMC_OK;
}

}  // namespace

int launch_match_filter(const int32_t* idx, const float* dist, const double* kp_tpl, const double* kp_q,
                        const int32_t* q_off, int n_frames, int n_tpl, double ratio, double d_lo, double d_hi,
                        double* kp_ordered, uint32_t* keep_bits, int32_t* counts, hipStream_t s) {
  int P = 1;
  while (P < n_tpl) P <<= 1;
  hipLaunchKernelGGL(match_filter_kernel, dim3(n_frames), dim3(kFilterThreads), (size_t)P * sizeof(double), s, idx,
                     dist, kp_tpl, kp_q, q_off, n_tpl, ratio, d_lo, d_hi, kp_ordered, keep_bits, counts);
  return launch_check("match_filter_kernel");
}

}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_knn2_l2u8(kcmc_ctx* ctx, const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q,
                              const int32_t* q_off, int n_frames, int max_nq, int32_t* out_idx,
                              float* out_dist, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_knn2_l2u8: ctx is NULL");
  KCMC_TRY(check_match_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  return launch_knn(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist, (hipStream_t)stream);
}

extern "C" int kcmc_match_frames(kcmc_ctx* ctx, const uint8_t* des_tpl, const double* kp_tpl, int n_tpl, int D,
                                 const uint8_t* des_q, const double* kp_q, const int32_t* q_off, int n_frames,
                                 int max_nq, double ratio, double d_lo, double d_hi, int32_t* out_idx,
                                 float* out_dist, double* out_kp_ordered, uint32_t* out_keep_bits,
                                 int32_t* out_counts, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_match_frames: ctx is NULL");
  KCMC_TRY(check_match_args(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist));
  if (n_frames > 0 && n_tpl > 0 && (!kp_tpl || !out_kp_ordered || !out_keep_bits || !out_counts || (max_nq > 0 && !kp_q)))
    return fail(KCMC_EINVAL, "kcmc_match_frames: NULL pointer");
  if (n_tpl > 8192) return fail(KCMC_EUNSUPPORTED, "kcmc_match_frames: n_tpl > 8192");
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  hipStream_t s = (hipStream_t)stream;
  KCMC_TRY(launch_knn(des_tpl, n_tpl, D, des_q, q_off, n_frames, max_nq, out_idx, out_dist, s));
  return launch_match_filter(out_idx, out_dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio, d_lo, d_hi,
                             out_kp_ordered, out_keep_bits, out_counts, s);
}
