// K1: batched k=2 L2 matching of uint8 descriptors + the per-frame match filters.
//
// Reference: VA:194-214 (cv2.BFMatcher(crossCheck=False).knnMatch(des_template,
// des_query, k=2), best-match reorder, ratio filter, median displacement filter).
//
// knn2_l2u8_kernel -- persistent: a workgroup keeps 256 / 512 template rows in registers
//   and matches them against a strided set of frames.
//   The distance is an exact integer contraction, so it runs on the int8 matrix
//   cores.  With x = a - 128 (template) and y = 127 - b (frame), both int8,
//   a - b = x + y + 1, so SSD = T + Q + 2 x.y with T = sum(x^2 + 2x) + D per template
//   row and Q = sum(y^2 + 2y) per frame row.  One v_mfma_i32_32x32x32_i8 pass per
//   32-deep k-step gives x.y (accumulator from zero).  T is constant along a template
//   column, so a column's frame rows are ordered by SSD - T + B = Q + 2 x.y + B, with
//   B = 2^20 = max T; the key is non-negative because SSD >= 0 (and < 2^23).  A operand = 32 frame
//   descriptors (rows j), B operand = 32 template descriptors (columns i): each lane
//   owns one template column and 16 frame rows of the 32x32 tile and keeps a running
//   top-2 in registers.
//   The top-2 runs on 32-bit keys ((SSD - T + B) << 8 | j - q0) local to a 256-row
//   chunk of frame descriptors: for D <= 64 bytes sqrtf is strictly increasing on the
//   integer SSD range, so integer keys order exactly like OpenCV's float
//   distances, and the low bits make ties go to the lower frame index like OpenCV's
//   K-insertion.  2.5 VALU ops per distance (the kernel is bound by integer VALU issue,
//   4 cycles per wave64 op): key = acc << 9 + qk (v_lshl_add, qk = (Q + B) << 8 | j - q0
//   from LDS) for two rows of a column, then b2 = min(b2, med3(b1, ka, kb)),
//   b1 = min3(b1, ka, kb), on two independent top-2 pairs per column so that consecutive
//   pairs do not wait on each other.  Each chunk's top-2 is merged into a 64-bit
//   (ssd << 32 | j) top-2 with SSD = (key >> 8) + T - B.  Frame descriptors are staged
//   through LDS (converted to int8, zero-padded to DP, rows padded by 16 B so the
//   ds_read_b128 fragment reads are bank-conflict free).
//
// match_filter_kernel -- one workgroup per frame: VA:196-214 in float64 with the
//   reference's exact operation order (no FMA contraction; file built with
//   -ffp-contract=off), median by an LDS bitonic sort.
#include <cfloat>
#include <climits>

#include <atomic>

#include "kcmc_internal.h"

namespace kcmc {

// CU count of the calling thread's current device, cached per device id.
int device_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  int cus = cache[dev].load(std::memory_order_relaxed);
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev].store(cus, std::memory_order_relaxed);
  }
  return cus;
}

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kBlocksPerWave = 2;                         // 32-row template blocks per wave
template <int WAVES>
struct KnnShape {
  static constexpr int kThreads = 64 * WAVES;
  static constexpr int kTplPerWG = WAVES * kBlocksPerWave * 32;  // template rows per workgroup
};
constexpr int kQChunk = 256;                              // frame descriptors per LDS chunk (8-bit local index)
constexpr uint32_t kNoKey = 0xffffffffu;                  // chunk keys of real rows are < 2^31
constexpr uint32_t kPad = 0xc0000000u;                    // key of the padding rows of a tile (acc = 0)
// Bias of the frame-row term: B = 2^20 = max T (T = sum (x + 1)^2 over D <= 64 bytes with
// x = a - 128 in [-128, 127]: 64 * 128^2).  The biased keys stay >= 0 only because the SSD
// they encode is >= 0; the asserts keep every real key below the padding key.
constexpr int kBias = 1 << 20;
static_assert(64 * 128 * 128 <= kBias, "kBias must cover the largest template term T");
static_assert(((64ull * 255 * 255) << 8 | 0xffull) < kPad, "real keys (SSD << 8 | row) must stay below kPad");
constexpr unsigned long long kNoKey64 = ~0ull;

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// b1 <= b2 always; new b2 = median(b1, b2, key), new b1 = min(b1, key).
__device__ __forceinline__ void top2_insert(uint32_t& b1, uint32_t& b2, uint32_t key) {
  b2 = med3_u32(b1, b2, key);
  b1 = b1 < key ? b1 : key;
}

// two keys at once (3 ops): the second smallest of {b1, b2, ka, kb} is
// min(b2, median(b1, ka, kb)) because b2 >= b1.  Exact when the keys are distinct or
// equal keys are interchangeable (the per-chunk keys carry their row).
__device__ __forceinline__ void top2_insert2(uint32_t& b1, uint32_t& b2, uint32_t ka, uint32_t kb) {
  const uint32_t m = med3_u32(b1, ka, kb);
  b1 = min3_u32(b1, ka, kb);
  b2 = b2 < m ? b2 : m;
}

__device__ __forceinline__ void top2_insert64(unsigned long long& b1, unsigned long long& b2, unsigned long long key) {
  const unsigned long long hi = b1 > key ? b1 : key;
  b2 = b2 < hi ? b2 : hi;
  b1 = b1 < key ? b1 : key;
}

// 4 consecutive descriptor bytes at column `col`, each XORed with `x` (0x80: a - 128,
// 0x7f: 127 - b as int8), zero past D.
__device__ __forceinline__ uint32_t load4_xor(const uint8_t* row, int col, int D, uint32_t x) {
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    uint32_t v = (col + b < D) ? (uint32_t)(row[col + b] ^ x) : 0u;
    w |= v << (8 * b);
  }
  return w;
}

// sum(v^2 + 2v) over the four int8 lanes of w, accumulated into acc
__device__ __forceinline__ int sq2(uint32_t w, int acc) {
  acc = __builtin_amdgcn_sdot4((int)w, (int)w, acc, false);
  return __builtin_amdgcn_sdot4((int)w, 0x02020202, acc, false);
}

// Chunk staging, one frame descriptor row per thread (row q0 + tid of a 256-row chunk):
// 16-byte loads at offsets 0, 16, ... of the row (rows are not 16-byte aligned unless
// D % 16 == 0; unaligned global loads are allowed), the last one running up to 15 bytes
// into the next row (masked off when landing).  Only the very last row of des_q would run
// past the buffer: its tail is read bytewise.  The loads of the next chunk are issued
// before the current chunk's MFMA tiles so that their latency hides behind them.
// Landing turns them into the padded int8 row (127 - b, zero past D), its key part
// (Q + B) << 8 | row and the LDS writes, all in registers.
template <int DP>
struct RowPieces {
  static constexpr int kNP = DP / 16;
};

__device__ __forceinline__ uint4 load16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);  // global_load_dwordx4 (unaligned access is allowed for global memory)
  return v;
}

template <int DP>
__device__ __forceinline__ void issue_row(const uint8_t* __restrict__ row, int D, bool last_row,
                                          uint4 (&pf)[RowPieces<DP>::kNP]) {
  constexpr int NP = RowPieces<DP>::kNP;
  const int np = (D + 15) >> 4;  // pieces holding the row (uniform)
#pragma unroll
  for (int k = 0; k < NP; ++k) pf[k] = load16(row + 16 * min(k, np - 1));
  if (last_row && (D & 15) != 0) {  // one lane in the whole grid: no read past des_q
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (16 * (np - 1) + c < D) w[c >> 2] |= (uint32_t)row[16 * (np - 1) + c] << (8 * (c & 3));
#pragma unroll
    for (int k = 0; k < NP; ++k)  // (a register array is never indexed at run time)
      if (k == np - 1) pf[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// mask of the bytes of word `w` (0..3) of piece `k` that lie inside the descriptor
__device__ __forceinline__ uint32_t byte_mask(int D, int k, int w) {
  const int n = D - 16 * k - 4 * w;  // bytes of this word inside the row
  return n >= 4 ? ~0u : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
}

template <int DP>
__device__ __forceinline__ void land_row(uint8_t* qrow, uint32_t* qk, int r, bool real, int D,
                                         const uint4 (&pf)[RowPieces<DP>::kNP]) {
  int nb = kBias;
#pragma unroll
  for (int k = 0; k < RowPieces<DP>::kNP; ++k) {
    uint4 v = pf[k];
    // int8 127 - b inside the row, zero past D (the masks are uniform)
    v.x = (v.x ^ 0x7f7f7f7fu) & byte_mask(D, k, 0);
    v.y = (v.y ^ 0x7f7f7f7fu) & byte_mask(D, k, 1);
    v.z = (v.z ^ 0x7f7f7f7fu) & byte_mask(D, k, 2);
    v.w = (v.w ^ 0x7f7f7f7fu) & byte_mask(D, k, 3);
    if (!real) v = make_uint4(0u, 0u, 0u, 0u);
    nb = sq2(v.x, nb);
    nb = sq2(v.y, nb);
    nb = sq2(v.z, nb);
    nb = sq2(v.w, nb);
    *reinterpret_cast<uint4*>(qrow + 16 * k) = v;
  }
  // padding rows of the last tile (zero descriptors, so acc = 0) get the key kPad
  *qk = real ? (((uint32_t)nb << 8) | (uint32_t)r) : kPad;
}

// Persistent, template-stationary: workgroup (tg, g) keeps template rows
// [tg * kTplPerWG, +kTplPerWG) in registers for the whole launch and walks frames g,
// g + G, g + 2G, ... (G workgroups per template group), so the template is loaded once per
// workgroup instead of once per frame, and the loads of the next 256-row chunk -- which
// may be the next frame's first -- are in flight while the current chunk is matched.
// WAVES = 8: 512 template rows share each staged chunk (n_tpl > 256); WAVES = 4 otherwise.
template <int DP, int WAVES>
__global__ __launch_bounds__(KnnShape<WAVES>::kThreads) void knn2_l2u8_kernel(
    const uint8_t* __restrict__ des_tpl, int n_tpl, int D, const uint8_t* __restrict__ des_q,
    const int32_t* __restrict__ q_off, int n_frames, int n_tg, int32_t* __restrict__ out_idx,
    float* __restrict__ out_dist) {
  constexpr int KSTEPS = DP / 32;
  constexpr int ROWB = DP + 16;  // padded LDS row stride (bytes)
  // double-buffered chunks: one barrier per chunk (a wave writes chunk c + 1 only after
  // every wave has passed the barrier of chunk c, i.e. finished chunk c - 1)
  __shared__ __attribute__((aligned(16))) uint8_t qbuf[2][kQChunk * ROWB];
  __shared__ __attribute__((aligned(16))) uint32_t qkey[2][kQChunk];

  // the template groups of a frame get consecutive ids of one XCD's run: they stage the
  // same frame rows, which then stay in that XCD's L2
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int tg = id % n_tg, g = id / n_tg, G = gridDim.x / n_tg;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c = lane & 31;   // MFMA column (template row within a block)
  const int h = lane >> 5;   // k-half of the fragment / row group of the output
  const int last_global = q_off[n_frames] - 1;  // des_q's last row

  // ---- template fragments (B operand) and T = sum(x^2 + 2x) + D, kept in registers
  v4i bfrag[kBlocksPerWave][KSTEPS];
  int tk[kBlocksPerWave];
  int tpl_row[kBlocksPerWave];
#pragma unroll
  for (int b = 0; b < kBlocksPerWave; ++b) {
    const int i = tg * KnnShape<WAVES>::kTplPerWG + (wave * kBlocksPerWave + b) * 32 + c;
    tpl_row[b] = i;
    int na = 0;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      if (i < n_tpl) {
        const uint8_t* row = des_tpl + (size_t)i * D;
#pragma unroll
        for (int d = 0; d < 4; ++d) w[d] = load4_xor(row, 32 * kk + 16 * h + 4 * d, D, 0x80u);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) na = sq2(w[d], na);
      bfrag[b][kk] = v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    }
    na += __shfl_xor(na, 32);
    tk[b] = na + D;
  }

  // ---- the item sequence: the 256-row chunks of frames g, g + G, ... that have rows
  // (a frame without rows still gets its epilogue).  nxt = the item whose loads are in
  // flight: frame nf, first row nq0 (nf >= n_frames: none).
  auto advance = [&](int f, int q0) -> int2 {  // the item after (f, q0)
    if (q0 + kQChunk < q_off[f + 1] - q_off[f]) return make_int2(f, q0 + kQChunk);
    for (f += G; f < n_frames && q_off[f + 1] == q_off[f]; f += G) {
    }
    return make_int2(f, 0);
  };
  auto issue = [&](int2 it, uint4 (&pf)[RowPieces<DP>::kNP]) {
    if (it.x < n_frames && tid < kQChunk) {
      const int qb = q_off[it.x], nq = q_off[it.x + 1] - qb;
      const int r = qb + it.y + min(tid, nq - it.y - 1);
      issue_row<DP>(des_q + (size_t)r * D, D, r == last_global, pf);
    }
  };
  uint4 pf[RowPieces<DP>::kNP];
  int2 nxt = make_int2(g, 0);  // the first item: frame g's first chunk, or the next frame with rows
  if (g < n_frames && q_off[g + 1] == q_off[g]) nxt = advance(g, 0);
  issue(nxt, pf);
  int buf = 0;
  for (int f = g; f < n_frames; f += G) {
    const int n_q = q_off[f + 1] - q_off[f];
    unsigned long long g1[kBlocksPerWave], g2[kBlocksPerWave];
#pragma unroll
    for (int b = 0; b < kBlocksPerWave; ++b) g1[b] = g2[b] = kNoKey64;
    for (int q0 = 0; q0 < n_q; q0 += kQChunk, buf ^= 1) {
      const int cnt = min(kQChunk, n_q - q0);
      const int rows = (cnt + 31) & ~31;
      // ---- stage frame descriptors [q0, q0+cnt) as int8 127 - b, zero-padded to DP columns
      if (tid < rows) land_row<DP>(&qbuf[buf][tid * ROWB], &qkey[buf][tid], tid, tid < cnt, D, pf);
      __syncthreads();
      nxt = advance(f, q0);
      issue(nxt, pf);
      const uint8_t* qb = qbuf[buf];
      const uint32_t* qkb = qkey[buf];
      uint32_t b1[kBlocksPerWave][2], b2[kBlocksPerWave][2];  // [even | odd accumulator]
#pragma unroll
      for (int b = 0; b < kBlocksPerWave; ++b) b1[b][0] = b2[b][0] = b1[b][1] = b2[b][1] = kNoKey;
      // ---- MFMA tiles of 32 frame rows
      for (int t0 = 0; t0 < rows; t0 += 32) {
        v4i afrag[KSTEPS];
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk)
          afrag[kk] = *reinterpret_cast<const v4i*>(&qb[(t0 + c) * ROWB + 32 * kk + 16 * h]);
        // rows of this lane's 16 accumulators: t0 + (r&3) + 8*(r>>2) + 4*h
        uint32_t qk[16];
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) qk[4 * gg + s2] = qkb[t0 + 8 * gg + 4 * h + s2];
        // every block's MFMAs first, so that block b + 1's matrix work overlaps block b's
        // top-2 epilogue instead of the epilogue waiting out each chain's latency
        v16i acc[kBlocksPerWave];
#pragma unroll
        for (int b = 0; b < kBlocksPerWave; ++b) {
          acc[b] = v16i{};
#pragma unroll
          for (int kk = 0; kk < KSTEPS; ++kk)  // acc = x.y
            acc[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag[kk], bfrag[b][kk], acc[b], 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < kBlocksPerWave; ++b)
#pragma unroll
          for (int p = 0; p < 8; ++p)
            top2_insert2(b1[b][p & 1], b2[b][p & 1], ((uint32_t)acc[b][2 * p] << 9) + qk[2 * p],
                         ((uint32_t)acc[b][2 * p + 1] << 9) + qk[2 * p + 1]);
      }
      // ---- fold the chunk's top-2 (local indices) into the frame's 64-bit top-2: the
      // even / odd pairs merge in 32 bits first (c1 <= c2 = the chunk's two smallest keys)
#pragma unroll
      for (int b = 0; b < kBlocksPerWave; ++b) {
        const uint32_t c1 = min(b1[b][0], b1[b][1]);
        const uint32_t c2 = min(max(b1[b][0], b1[b][1]), min(b2[b][0], b2[b][1]));
        const uint32_t ks[2] = {c1, c2};
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (ks[k] < kPad) {
            const uint32_t ssd = (ks[k] >> 8) + (uint32_t)(tk[b] - kBias);
            top2_insert64(g1[b], g2[b], ((unsigned long long)ssd << 32) | (uint32_t)(q0 + (int)(ks[k] & 255u)));
          }
      }
    }
    // ---- merge the two row halves (lanes l and l^32 own the same template column)
#pragma unroll
    for (int b = 0; b < kBlocksPerWave; ++b) {
      const unsigned long long o1 = (unsigned long long)__shfl_xor((long long)g1[b], 32);
      const unsigned long long o2 = (unsigned long long)__shfl_xor((long long)g2[b], 32);
      unsigned long long m1 = g1[b], m2 = g2[b];
      top2_insert64(m1, m2, o1);
      top2_insert64(m1, m2, o2);
      const int i = tpl_row[b];
      if (h == 0 && i < n_tpl) {
        const size_t o = ((size_t)f * n_tpl + i) * 2;
        const unsigned long long ms[2] = {m1, m2};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          if (ms[k] == kNoKey64) {
            out_idx[o + k] = -1;
            out_dist[o + k] = FLT_MAX;
          } else {
            out_idx[o + k] = (int32_t)(ms[k] & 0xffffffffull);
            out_dist[o + k] = sqrtf((float)(ms[k] >> 32));
          }
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

// The same filters for n_tpl <= 512 with ONE wave per frame and no barrier: template i =
// 64 k + lane sits in the lane's register k (k < 8), and the median of the ratio survivors
// comes from a bitonic sort of all 512 register slots (non-survivors +inf) across the wave
// (stride < 8: within a lane; >= 8: shuffles with lane ^ stride / 8), so the survivors need
// no compaction: the sorted slots 0 .. nr - 1 are their sorted displacements.  The
// barrier-per-stage sort of the workgroup kernel waited ~40 us per launch at c2 / c3.
constexpr int kFilterWaveFrames = 4;  // frames (waves) per 256-thread workgroup

__device__ __forceinline__ void cmpx(double& a, double& b, bool asc) {
  const double lo = fmin(a, b), hi = fmax(a, b);
  a = asc ? lo : hi;
  b = asc ? hi : lo;
}

__global__ __launch_bounds__(64 * kFilterWaveFrames) void match_filter_wave_kernel(
    const int32_t* __restrict__ idx, const float* __restrict__ dist, const double* __restrict__ kp_tpl,
    const double* __restrict__ kp_q, const int32_t* __restrict__ q_off, int n_frames, int n_tpl, double ratio,
    double d_lo, double d_hi, double* __restrict__ kp_ordered, uint32_t* __restrict__ keep_bits,
    int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * kFilterWaveFrames + (threadIdx.x >> 6);
  if (f >= n_frames) return;  // the whole wave
  const int q_begin = q_off[f];
  const int words = (n_tpl + 31) >> 5;
  // pass 1: reorder (VA:197-200), ratio filter (VA:202-203), displacement of survivors (VA:208)
  double dv[8];
  uint64_t okm[8];
  int nr = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = 64 * k + lane;
    bool ok = false;
    double d = INFINITY;
    if (i < n_tpl) {
      const size_t o = ((size_t)f * n_tpl + i) * 2;
      const int j0 = idx[o];
      double qx = 0.0, qy = 0.0;
      if (j0 >= 0) {
        qx = kp_q[2 * (size_t)(q_begin + j0)];
        qy = kp_q[2 * (size_t)(q_begin + j0) + 1];
      }
      kp_ordered[((size_t)f * n_tpl + i) * 2] = qx;
      kp_ordered[((size_t)f * n_tpl + i) * 2 + 1] = qy;
      ok = (double)dist[o] < ratio * (double)dist[o + 1];
      if (ok) {
        const double dx = kp_tpl[2 * i] - qx, dy = kp_tpl[2 * i + 1] - qy;
        d = sqrt(dx * dx + dy * dy);
      }
    }
    dv[k] = d;
    okm[k] = __ballot(ok);
    nr += __popcll(okm[k]);
  }
  // bitonic sort (ascending) of the 512 slots e = 8 lane + k
  double v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = dv[k];
#pragma unroll
  for (int size = 2; size <= 512; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 8) {
        const int ls = stride >> 3;
        const bool lower = (lane & ls) == 0;
        const bool asc = size >= 16 ? (lane & (size >> 3)) == 0 : true;  // (e & size) == 0
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double o = __shfl_xor(v[k], ls, 64);
          v[k] = (lower == asc) ? fmin(v[k], o) : fmax(v[k], o);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if ((k & stride) == 0) {
            const bool asc = size >= 8 ? (lane & (size >> 3)) == 0 : (k & size) == 0;  // (e & size) == 0
            cmpx(v[k], v[k | stride], asc);
          }
        }
      }
    }
  }
  // the median of the nr survivors: sorted slots (nr - 1) / 2 and nr / 2 (np.median, VA:210)
  double med = 0.0;
  if (nr > 0) {
    auto slot = [&](int e) -> double {
      double x = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if ((e & 7) == k) x = v[k];  // wave-uniform
      return __shfl(x, e >> 3, 64);
    };
    const double b = slot(nr >> 1);
    med = (nr & 1) ? b : (slot((nr >> 1) - 1) + b) / 2.0;
  }
  const double lo = d_lo * med, hi = d_hi * med;
  // pass 2: keep = ratio survivor and lo <= d <= hi (VA:210); bitmask + counts
  int nk = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool keep = nr > 0 && ((okm[k] >> lane) & 1ull) && lo <= dv[k] && dv[k] <= hi;
    const uint64_t m = __ballot(keep);
    nk += __popcll(m);
    if (lane == 0) {
      if (2 * k < words) keep_bits[(size_t)f * words + 2 * k] = (uint32_t)m;
      if (2 * k + 1 < words) keep_bits[(size_t)f * words + 2 * k + 1] = (uint32_t)(m >> 32);
    }
  }
  if (lane == 0) {
    counts[4 * (size_t)f + 0] = n_tpl;  // len(kp_query) after the reorder at VA:200
    counts[4 * (size_t)f + 1] = n_tpl;  // len(matches)
    counts[4 * (size_t)f + 2] = nr;
    counts[4 * (size_t)f + 3] = nk;
  }
}

// The same for 512 < n_tpl <= 4096: one 512-thread workgroup per frame, template
// i = 512 k + tid in register k of thread tid, and a 4096-slot bitonic sort (slot
// e = 8 tid + k): strides < 8 within a thread, < 512 by shuffles inside a wave, and only
// the strides 512..2048 (6 of the 78 stages) through LDS with barriers (the workgroup
// kernel above synchronises at all 78).
constexpr int kFilterWgThreads = 512;

__global__ __launch_bounds__(kFilterWgThreads) void match_filter_wg_kernel(
    const int32_t* __restrict__ idx, const float* __restrict__ dist, const double* __restrict__ kp_tpl,
    const double* __restrict__ kp_q, const int32_t* __restrict__ q_off, int n_tpl, double ratio, double d_lo,
    double d_hi, double* __restrict__ kp_ordered, uint32_t* __restrict__ keep_bits, int32_t* __restrict__ counts) {
  __shared__ double sx[kFilterWgThreads * 8];
  __shared__ int s_cnt[kFilterWgThreads / 64];
  __shared__ double s_med[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int f = blockIdx.x;
  const int q_begin = q_off[f];
  const int words = (n_tpl + 31) >> 5;
  double dv[8];
  uint64_t okm[8];
  int nr = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = kFilterWgThreads * k + tid;
    bool ok = false;
    double d = INFINITY;
    if (i < n_tpl) {
      const size_t o = ((size_t)f * n_tpl + i) * 2;
      const int j0 = idx[o];
      double qx = 0.0, qy = 0.0;
      if (j0 >= 0) {
        qx = kp_q[2 * (size_t)(q_begin + j0)];
        qy = kp_q[2 * (size_t)(q_begin + j0) + 1];
      }
      kp_ordered[((size_t)f * n_tpl + i) * 2] = qx;
      kp_ordered[((size_t)f * n_tpl + i) * 2 + 1] = qy;
      ok = (double)dist[o] < ratio * (double)dist[o + 1];
      if (ok) {
        const double dx = kp_tpl[2 * i] - qx, dy = kp_tpl[2 * i + 1] - qy;
        d = sqrt(dx * dx + dy * dy);
      }
    }
    dv[k] = d;
    okm[k] = __ballot(ok);
    nr += __popcll(okm[k]);
  }
  if (lane == 0) s_cnt[wave] = nr;
  __syncthreads();
  nr = 0;
#pragma unroll
  for (int w = 0; w < kFilterWgThreads / 64; ++w) nr += s_cnt[w];
  double v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = dv[k];
#pragma unroll
  for (int size = 2; size <= 8 * kFilterWgThreads; size <<= 1) {
    const bool asc_t = (tid & (size >> 3)) == 0;  // (e & size) == 0 for size >= 8
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 512) {  // partner in another wave: through LDS
        const int ts = stride >> 3;
        const bool lower = (tid & ts) == 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) sx[8 * tid + k] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double o = sx[8 * (tid ^ ts) + k];
          v[k] = (lower == asc_t) ? fmin(v[k], o) : fmax(v[k], o);
        }
        __syncthreads();
      } else if (stride >= 8) {
        const int ls = stride >> 3;
        const bool lower = (tid & ls) == 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double o = __shfl_xor(v[k], ls, 64);
          v[k] = (lower == asc_t) ? fmin(v[k], o) : fmax(v[k], o);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if ((k & stride) == 0) {
            const bool asc = size >= 8 ? asc_t : (k & size) == 0;
            cmpx(v[k], v[k | stride], asc);
          }
        }
      }
    }
  }
  // the median of the nr survivors: sorted slots (nr - 1) / 2 and nr / 2 (np.median, VA:210)
  if (nr > 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = 8 * tid + k;
      if (e == (nr >> 1)) s_med[1] = v[k];
      if ((nr & 1) == 0 && e == (nr >> 1) - 1) s_med[0] = v[k];
    }
  }
  __syncthreads();
  double med = 0.0;
  if (nr > 0) med = (nr & 1) ? s_med[1] : (s_med[0] + s_med[1]) / 2.0;
  const double lo = d_lo * med, hi = d_hi * med;
  int nk = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool keep = nr > 0 && ((okm[k] >> lane) & 1ull) && lo <= dv[k] && dv[k] <= hi;
    const uint64_t m = __ballot(keep);
    nk += __popcll(m);
    const int w0 = (kFilterWgThreads * k + 64 * wave) >> 5;
    if (lane == 0) {
      if (w0 < words) keep_bits[(size_t)f * words + w0] = (uint32_t)m;
      if (w0 + 1 < words) keep_bits[(size_t)f * words + w0 + 1] = (uint32_t)(m >> 32);
    }
  }
  __syncthreads();  // s_cnt is reused
  if (lane == 0) s_cnt[wave] = nk;
  __syncthreads();
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < kFilterWgThreads / 64; ++w) tot += s_cnt[w];
    counts[4 * (size_t)f + 0] = n_tpl;
    counts[4 * (size_t)f + 1] = n_tpl;
    counts[4 * (size_t)f + 2] = nr;
    counts[4 * (size_t)f + 3] = tot;
  }
}

// persistent grid: n_tg template groups x G frame strides, G = the resident workgroups
// per template group (workgroups never wait on each other, so a wrong residency count
// costs balance, not progress)
int knn_grid(int n_tg, int n_frames, int wgs_per_cu) {
  const int G = std::max(1, std::min(n_frames, device_cus() * std::max(1, wgs_per_cu) / n_tg));
  return n_tg * G;
}

template <typename K>
int resident_wgs(K kernel, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}

template <int DP, int WAVES>
int launch_knn_row(const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q, const int32_t* q_off,
                   int n_frames, int32_t* out_idx, float* out_dist, hipStream_t s) {
  auto* k = knn2_l2u8_kernel<DP, WAVES>;
  static const int per_cu = resident_wgs(k, KnnShape<WAVES>::kThreads);
  const int n_tg = ceil_div(n_tpl, KnnShape<WAVES>::kTplPerWG);
  hipLaunchKernelGGL(k, dim3(knn_grid(n_tg, n_frames, per_cu)), dim3(KnnShape<WAVES>::kThreads), 0, s, des_tpl,
                     n_tpl, D, des_q, q_off, n_frames, n_tg, out_idx, out_dist);
  return launch_check("knn2_l2u8_kernel");
}

int launch_knn(const uint8_t* des_tpl, int n_tpl, int D, const uint8_t* des_q, const int32_t* q_off,
               int n_frames, int max_nq, int32_t* out_idx, float* out_dist, hipStream_t s) {
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  (void)max_nq;
  const bool wide = n_tpl > 256;  // 512 template rows share each staged chunk
  if (D <= 32)
    return wide ? launch_knn_row<32, 8>(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s)
                : launch_knn_row<32, 4>(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s);
  return wide ? launch_knn_row<64, 8>(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s)
              : launch_knn_row<64, 4>(des_tpl, n_tpl, D, des_q, q_off, n_frames, out_idx, out_dist, s);
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
  if (n_tpl <= 512) {
    hipLaunchKernelGGL(match_filter_wave_kernel, dim3(ceil_div(n_frames, kFilterWaveFrames)),
                       dim3(64 * kFilterWaveFrames), 0, s, idx, dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio,
                       d_lo, d_hi, kp_ordered, keep_bits, counts);
    return launch_check("match_filter_wave_kernel");
  }
  if (n_tpl <= 8 * kFilterWgThreads) {
    hipLaunchKernelGGL(match_filter_wg_kernel, dim3(n_frames), dim3(kFilterWgThreads), 0, s, idx, dist, kp_tpl, kp_q,
                       q_off, n_tpl, ratio, d_lo, d_hi, kp_ordered, keep_bits, counts);
    return launch_check("match_filter_wg_kernel");
  }
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

extern "C" int kcmc_match_filter(kcmc_ctx* ctx, const int32_t* idx, const float* dist, const double* kp_tpl,
                                 const double* kp_q, const int32_t* q_off, int n_frames, int n_tpl, double ratio,
                                 double d_lo, double d_hi, double* out_kp_ordered, uint32_t* out_keep_bits,
                                 int32_t* out_counts, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_match_filter: ctx is NULL");
  if (n_tpl < 0 || n_frames < 0) return fail(KCMC_EINVAL, "kcmc_match_filter: negative size");
  if (n_frames > 65535) return fail(KCMC_EUNSUPPORTED, "kcmc_match_filter: at most 65535 frames per call");
  if (n_tpl > 8192) return fail(KCMC_EUNSUPPORTED, "kcmc_match_filter: n_tpl > 8192");
  if (n_frames == 0 || n_tpl == 0) return KCMC_OK;
  if (!idx || !dist || !kp_tpl || !kp_q || !q_off || !out_kp_ordered || !out_keep_bits || !out_counts)
    return fail(KCMC_EINVAL, "kcmc_match_filter: NULL pointer");
  return launch_match_filter(idx, dist, kp_tpl, kp_q, q_off, n_frames, n_tpl, ratio, d_lo, d_hi, out_kp_ordered,
                             out_keep_bits, out_counts, (hipStream_t)stream);
}
