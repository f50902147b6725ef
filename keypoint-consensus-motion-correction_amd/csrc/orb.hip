// f1: keypoint detection + description on the device.
//
// The reference detects with OpenCV AKAZE/BRISK in the host process and per joblib
// worker (VA:114-116, VA:190-192); BASELINE config 2 names ORB keypoints.  OpenCV is
// absent from this image, so the detector is build-defined -- an exact, integer,
// single-scale ORB-style detector (oracle: kcmc_oracle_orb_detect, bit-identical):
//   * FAST-9 score: the largest t for which 9 contiguous pixels of the radius-3 circle
//     are all brighter, or all darker, than the centre by more than t; a corner if
//     score > threshold;
//   * 3x3 non-maximum suppression on the score (ties: the first in raster order wins);
//   * Harris response of the survivors from integer Sobel sums over 7x7,
//     R = (ab - c^2) - k (a+b)^2 in double;
//   * the n_features largest R per frame (ties: candidate order), candidates ordered
//     by 64x16 tile (row-major) then raster order in the tile -- the output order;
//   * intensity-centroid orientation over the radius-15 disc, binned into 32 bins with
//     exact cross-product tests against the bin edges;
//   * steered BRIEF: 256 point pairs of a fixed pattern rotated to the bin's centre
//     angle (host table), compared on a 5x5 binomial smoothing -> 32-byte descriptors.
//
// orb_candidates_kernel  one workgroup per kSub vertically stacked 64x16 tiles: image +
//                        4-px halo in LDS, FAST scores for the region + 1-px halo, NMS,
//                        Harris -- each step on the compacted survivors of the previous
//                        one (block scans), so the candidates keep tile order and raster
//                        order inside the tile.
// orb_offsets_kernel +   per frame: tile prefix offsets, then one wave per tile copies
// orb_gather_kernel      its candidates into the frame's compact list (candidate order).
// orb_select_kernel      one workgroup per frame: radix select of the n_features-th
//                        largest key, ordered compaction of the kept candidates.
// orb_describe_kernel    one wave per keypoint: moments (wave reduction), bin, 4 x 64
//                        BRIEF comparisons of on-the-fly smoothed samples (ballots).
#include <cmath>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

constexpr int kThreads = 256;
constexpr int kTW = 64, kTH = 16;          // candidate tile (the candidate order's unit)
constexpr int kSub = 2;                    // tiles per workgroup, stacked vertically (4: slower)
constexpr int kRH = kTH * kSub;            // rows of a workgroup's region
constexpr int kHalo = 4;                   // FAST radius 3 + NMS 1; Harris 3 + Sobel 1
constexpr int kPW = kTW + 2 * kHalo;       // 72
constexpr int kPH = kRH + 2 * kHalo;
constexpr int kSW = kTW + 2, kSH = kRH + 2;  // scores of the region + 1-px halo
constexpr int kSlots = kTW * kTH / 4;      // per tile: NMS leaves at most one candidate per 2x2 block
constexpr int kNmsPx = kTW * kRH / kThreads;  // region pixels per thread in the NMS (one tile's run)
static_assert(kNmsPx <= 32 && (kTW * kTH) % kNmsPx == 0, "NMS: a thread's pixels lie in one tile");

__constant__ int8_t c_circle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                       {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

__device__ __forceinline__ uint64_t order_key(double r) {
  const uint64_t u = (uint64_t)__double_as_longlong(r);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

// Exclusive block scan of one int per thread (256 threads); returns the total.
__device__ __forceinline__ int block_excl_scan(int v, int* s_warp, int& excl) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_warp[wave] = x;
  __syncthreads();
  int base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    const int t = s_warp[w];
    if (w < wave) base += t;
    total += t;
  }
  __syncthreads();
  excl = base + x - v;
  return total;
}

// FAST-9 score of one pixel (max over the 16 contiguous 9-pixel arcs of the smaller
// threshold margin, positive or negative side): running minima over 2, 4, 8 then 9
// neighbours on the circle, both sides at once.
__device__ __forceinline__ int fast_score9(const uint8_t (*img)[kPW], int py, int px) {
  const int v = img[py][px];
  int d[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) d[j] = (int)img[py + c_circle[j][1]][px + c_circle[j][0]] - v;
  int lo2[16], hi2[16], lo4[16], hi4[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    lo2[j] = min(d[j], d[(j + 1) & 15]);
    hi2[j] = max(d[j], d[(j + 1) & 15]);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    lo4[j] = min(lo2[j], lo2[(j + 2) & 15]);
    hi4[j] = max(hi2[j], hi2[(j + 2) & 15]);
  }
  int best = -1000;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int mb = min(min(lo4[k], lo4[(k + 4) & 15]), d[(k + 8) & 15]);   // min of d over the arc
    const int Md = max(max(hi4[k], hi4[(k + 4) & 15]), d[(k + 8) & 15]);  // max of d over the arc
    best = max(best, max(mb, -Md));
  }
  return best;
}

// One workgroup per kSub vertically stacked 64x16 tiles (a 64 x kRH region: the barriers
// and the halo of one tile's worth of work are shared by kSub tiles).  Candidates are
// sparse, so every expensive step runs on a compacted list instead of on all pixels (a
// wave would otherwise pay for its single candidate with 63 idle lanes): (1) stage the
// image + 4-px halo; (2) the compass pre-test on the region + 1-px halo, survivors
// listed; (3) FAST scores of the listed pixels; (4) 3x3 NMS of the region's pixels,
// survivors listed in raster order -- which is tile order, then raster order inside the
// tile, the candidate order; (5) integer Harris of the listed candidates, 8 lanes per
// candidate (one 7-pixel window row each, shuffle reduction); (6) the keys and positions
// stored per tile, in list order.
// 8 waves per SIMD (<= 64 VGPRs, no spill): the workgroups are barrier- and latency-bound,
// and the eighth wave slot took 15.4 -> 14.8 ms per 2000 c2 frames (profiles/r06_orb_subtiles_ab.txt)
__global__ __launch_bounds__(kThreads, 8) void orb_candidates_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                                  int threshold, double harris_k, int edge,
                                                                  uint64_t* __restrict__ cand_key,
                                                                  uint32_t* __restrict__ cand_pos,
                                                                  int32_t* __restrict__ cand_cnt) {
  __shared__ __attribute__((aligned(16))) uint8_t img[kPH][kPW];
  __shared__ int16_t sc[kSH][kSW];
  __shared__ uint16_t plist[kSH * kSW];  // pre-test survivors (score-region index)
  __shared__ uint16_t nlist[kTW * kRH];  // NMS survivors (region pixel index, raster order)
  __shared__ int s_warp[kThreads / 64];
  __shared__ int s_start[kSub + 1];      // the first list entry of each tile; s_start[kSub] = total
  const int ntx = gridDim.x;
  const int nty = (H + kTH - 1) / kTH;   // tile rows of the frame (the last region may hold fewer)
  const int f = blockIdx.z;
  const int x0 = blockIdx.x * kTW, y0 = blockIdx.y * kRH;
  const int tid = threadIdx.x;
  const uint8_t* I = frames + (size_t)f * H * W;

  // (1) staging: 4-byte words where the row is aligned (x0 - 4 is a multiple of 4)
  if ((W & 3) == 0) {
    for (int i = tid; i < kPH * (kPW / 4); i += kThreads) {
      const int r = i / (kPW / 4), c = 4 * (i - r * (kPW / 4));
      const int y = y0 - kHalo + r, x = x0 - kHalo + c;
      uint32_t v = 0;
      if ((unsigned)y < (unsigned)H && x >= 0 && x + 4 <= W) v = *reinterpret_cast<const uint32_t*>(I + (size_t)y * W + x);
      *reinterpret_cast<uint32_t*>(&img[r][c]) = v;
    }
  } else {
    for (int i = tid; i < kPH * kPW; i += kThreads) {
      const int r = i / kPW, c = i - r * kPW;
      const int y = y0 - kHalo + r, x = x0 - kHalo + c;
      img[r][c] = ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) ? I[(size_t)y * W + x] : (uint8_t)0;
    }
  }
  __syncthreads();

  // (2) compass pre-test: a 9-pixel arc covers at least two of the four compass pixels
  // (0, 4, 8, 12), so fewer than two beyond the threshold on the same side -> score 0
  constexpr int kItems = (kSH * kSW + kThreads - 1) / kThreads;
  uint32_t pass = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int i = tid + kThreads * k;
    if (i >= kSH * kSW) break;
    const int r = i / kSW, c = i - r * kSW;
    const int y = y0 - 1 + r, x = x0 - 1 + c;
    sc[r][c] = 0;
    if (y >= 3 && y < H - 3 && x >= 3 && x < W - 3) {
      const int py = r - 1 + kHalo, px = c - 1 + kHalo;
      const int v = img[py][px];
      const int n0 = img[py + 3][px], n4 = img[py][px + 3], n8 = img[py - 3][px], n12 = img[py][px - 3];
      const int hi = (n0 > v + threshold) + (n4 > v + threshold) + (n8 > v + threshold) + (n12 > v + threshold);
      const int lo = (n0 < v - threshold) + (n4 < v - threshold) + (n8 < v - threshold) + (n12 < v - threshold);
      if (hi >= 2 || lo >= 2) pass |= 1u << k;
    }
  }
  int excl;
  const int npass = block_excl_scan(__builtin_popcount(pass), s_warp, excl);
#pragma unroll
  for (int k = 0; k < kItems; ++k)
    if (pass >> k & 1) plist[excl++] = (uint16_t)(tid + kThreads * k);
  __syncthreads();

  // (3) FAST scores of the listed pixels
  for (int j = tid; j < npass; j += kThreads) {
    const int i = plist[j];
    const int r = i / kSW, c = i - r * kSW;
    const int s = fast_score9(img, r - 1 + kHalo, c - 1 + kHalo);
    sc[r][c] = (int16_t)(s > threshold ? s : 0);
  }
  __syncthreads();

  // (4) NMS; thread t owns region pixels kNmsPx t .. kNmsPx t + kNmsPx - 1 (raster order),
  // all in tile kNmsPx t / 1024
  uint32_t flags = 0;
#pragma unroll
  for (int q = 0; q < kNmsPx; ++q) {
    const int p = kNmsPx * tid + q;
    const int r = p / kTW, c = p - r * kTW;
    const int y = y0 + r, x = x0 + c;
    if (y < edge || y >= H - edge || x < edge || x >= W - edge) continue;
    const int s = sc[r + 1][c + 1];
    if (s == 0) continue;
    bool keep = true;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        if (dx == 0 && dy == 0) continue;
        const int o = sc[r + 1 + dy][c + 1 + dx];
        const bool later = dy > 0 || (dy == 0 && dx > 0);
        keep = keep && (s > o || (s == o && later));
      }
    if (keep) flags |= 1u << q;
  }
  const int total = block_excl_scan(__builtin_popcount(flags), s_warp, excl);
  if ((kNmsPx * tid) % (kTW * kTH) == 0) s_start[kNmsPx * tid / (kTW * kTH)] = excl;  // a tile's first thread
  if (tid == 0) s_start[kSub] = total;
#pragma unroll
  for (int q = 0; q < kNmsPx; ++q)
    if (flags >> q & 1) nlist[excl++] = (uint16_t)(kNmsPx * tid + q);
  __syncthreads();

  // (5) Harris over the 7x7 window of Sobel gradients, 8 lanes per candidate (lane row
  // 0..6 sums its window row, lane 7 idles), then (6) the stores in list order
  const int grp = tid >> 3, row = tid & 7;
  for (int j0 = 0; j0 < total; j0 += kThreads / 8) {
    const int j = j0 + grp;
    int a = 0, b = 0, cc = 0;
    int p = 0;
    if (j < total) {
      p = nlist[j];
      if (row < 7) {
        const int r = p / kTW, c = p - r * kTW;
        const int py = r + kHalo + row - 3;
#pragma unroll
        for (int dx = -3; dx <= 3; ++dx) {
          const int px = c + kHalo + dx;
          const int ix = ((int)img[py - 1][px + 1] + 2 * (int)img[py][px + 1] + (int)img[py + 1][px + 1]) -
                         ((int)img[py - 1][px - 1] + 2 * (int)img[py][px - 1] + (int)img[py + 1][px - 1]);
          const int iy = ((int)img[py + 1][px - 1] + 2 * (int)img[py + 1][px] + (int)img[py + 1][px + 1]) -
                         ((int)img[py - 1][px - 1] + 2 * (int)img[py - 1][px] + (int)img[py - 1][px + 1]);
          a += ix * ix;  // |ix|, |iy| <= 1020: 49 terms stay below 2^31
          b += iy * iy;
          cc += ix * iy;
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      a += __shfl_xor(a, o);
      b += __shfl_xor(b, o);
      cc += __shfl_xor(cc, o);
    }
    if (j < total && row == 0) {
      const long long A = a, B = b, C = cc;
      const double sab = (double)(A + B);
      const int r = p / kTW, c = p - r * kTW;
      const int st = r / kTH;  // the candidate's tile in the region
      const size_t o = ((size_t)f * nty * ntx + (size_t)(blockIdx.y * kSub + st) * ntx + blockIdx.x) * kSlots +
                       (j - s_start[st]);
      cand_key[o] = order_key((double)(A * B - C * C) - harris_k * (sab * sab));
      cand_pos[o] = ((uint32_t)(y0 + r) << 16) | (uint32_t)(x0 + c);
    }
  }
  if (tid < kSub && blockIdx.y * kSub + tid < nty)
    cand_cnt[(size_t)f * nty * ntx + (size_t)(blockIdx.y * kSub + tid) * ntx + blockIdx.x] = s_start[tid + 1] - s_start[tid];
}

// Per frame, one wave per tile (in tile order): the tile's candidates are appended to
// the frame's compact list at the tile's prefix offset, keeping candidate order.
__global__ __launch_bounds__(kThreads) void orb_gather_kernel(const uint64_t* __restrict__ cand_key,
                                                              const uint32_t* __restrict__ cand_pos,
                                                              const int32_t* __restrict__ cand_cnt,
                                                              const int32_t* __restrict__ tile_off, int ntiles,
                                                              uint64_t* __restrict__ list_key,
                                                              uint32_t* __restrict__ list_pos) {
  const int f = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const size_t fb = (size_t)f * ntiles;
  for (int t = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); t < ntiles; t += gridDim.x * (kThreads / 64)) {
    const int cnt = cand_cnt[fb + t];
    const int off = tile_off[fb + t];
    for (int s = lane; s < cnt; s += 64) {
      list_key[fb * kSlots + off + s] = cand_key[(fb + t) * kSlots + s];
      list_pos[fb * kSlots + off + s] = cand_pos[(fb + t) * kSlots + s];
    }
  }
}

// Per frame (one workgroup): exclusive prefix of the tile counts -> tile offsets, total.
__global__ __launch_bounds__(kThreads) void orb_offsets_kernel(const int32_t* __restrict__ cand_cnt, int ntiles,
                                                               int32_t* __restrict__ tile_off,
                                                               int32_t* __restrict__ total) {
  __shared__ int s_warp[kThreads / 64];
  const int f = blockIdx.x;
  int carry = 0;
  for (int t0 = 0; t0 < ntiles; t0 += kThreads) {
    const int t = t0 + threadIdx.x;
    const int c = t < ntiles ? cand_cnt[(size_t)f * ntiles + t] : 0;
    int ex;
    const int tot = block_excl_scan(c, s_warp, ex);
    if (t < ntiles) tile_off[(size_t)f * ntiles + t] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) total[f] = carry;
}

// One workgroup per frame: the n_features-th largest key T of the compact list by 8-bit
// radix select, then the kept candidates (key > T, and the first ties) compacted in
// list order.
__global__ __launch_bounds__(kThreads) void orb_select_kernel(const uint64_t* __restrict__ list_key,
                                                              const uint32_t* __restrict__ list_pos,
                                                              const int32_t* __restrict__ total_n, int ntiles,
                                                              int n_features, double* __restrict__ out_kp,
                                                              uint32_t* __restrict__ out_pos,
                                                              int32_t* __restrict__ out_n, int f_base) {
  __shared__ int hist[256];
  __shared__ int s_warp[kThreads / 64];
  __shared__ uint64_t s_prefix;
  __shared__ int s_rank;
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t* K = list_key + (size_t)f * ntiles * kSlots;
  const uint32_t* Pp = list_pos + (size_t)f * ntiles * kSlots;
  const int total = total_n[f];
  const bool all = total <= n_features;
  uint64_t T = 0;
  int n_gt = 0;
  if (!all) {
    if (tid == 0) {
      s_prefix = 0;
      s_rank = n_features;
    }
    for (int d = 7; d >= 0; --d) {
      hist[tid] = 0;
      __syncthreads();
      const uint64_t prefix = s_prefix;
      const uint64_t hmask = d == 7 ? 0ull : (~0ull << (8 * (d + 1)));
      for (int i = tid; i < total; i += kThreads) {
        const uint64_t k = K[i];
        if ((k & hmask) == prefix) atomicAdd(&hist[(k >> (8 * d)) & 255], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int rank = s_rank, acc = 0, dig = 255;
        for (; dig > 0; --dig) {
          if (acc + hist[dig] >= rank) break;
          acc += hist[dig];
        }
        s_rank = rank - acc;
        s_prefix = prefix | ((uint64_t)dig << (8 * d));
      }
      __syncthreads();
    }
    T = s_prefix;
    n_gt = n_features - s_rank;  // keys strictly above T
  }
  int out = 0, ties = 0;
  for (int i0 = 0; i0 < total; i0 += kThreads) {
    const int i = i0 + tid;
    int keep = 0, tie = 0;
    if (i < total) {
      const uint64_t k = K[i];
      keep = all || k > T;
      tie = !all && k == T;
    }
    int tie_ex;
    const int tie_tot = block_excl_scan(tie, s_warp, tie_ex);
    if (tie && ties + tie_ex < n_features - n_gt) keep = 1;
    int ex;
    const int kept = block_excl_scan(keep, s_warp, ex);
    if (keep) {
      const uint32_t pp = Pp[i];
      const size_t o = (size_t)(f_base + f) * n_features + out + ex;
      out_pos[o] = pp;
      out_kp[2 * o] = (double)(pp & 0xffffu);
      out_kp[2 * o + 1] = (double)(pp >> 16);
    }
    out += kept;
    ties += tie_tot;
  }
  if (tid == 0) out_n[f_base + f] = out;
}

// The keypoint's 31x31 patch in LDS: moments use the radius-15 disc, BRIEF samples lie
// within radius 13 of the keypoint and their 5x5 smoothing adds 2.
constexpr int kPatch = 31, kPatchWords = 9;  // rows of 36 bytes from the 4-aligned column

__device__ __forceinline__ int patch_at(const uint8_t* P, int ofs, int dx, int dy) {
  return P[(dy + 15) * (4 * kPatchWords) + ofs + dx + 15];
}

// 5x5 binomial smoothing at one patch point: (sum w_i w_j I + 128) >> 8, w = 1 4 6 4 1.
__device__ __forceinline__ int smooth5_patch(const uint8_t* P, int ofs, int dx, int dy) {
  int s = 0;
  const int w[5] = {1, 4, 6, 4, 1};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint8_t* row = P + (dy + i - 2 + 15) * (4 * kPatchWords) + ofs + dx - 2 + 15;
    s += w[i] * ((int)row[0] + 4 * (int)row[1] + 6 * (int)row[2] + 4 * (int)row[3] + (int)row[4]);
  }
  return (s + 128) >> 8;
}

// One wave per keypoint: the 31x31 patch is staged into the wave's LDS slice with
// coalesced 4-byte loads (scattered byte loads of the patch kept the texture units busy
// for ~3400 cycles per keypoint), then intensity-centroid moments (wave reduction),
// exact bin, and 4 x 64 BRIEF comparisons of smoothed samples packed with ballots.
__global__ __launch_bounds__(kThreads) void orb_describe_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                                const uint32_t* __restrict__ kp_pos,
                                                                const int32_t* __restrict__ kp_n, int n_features,
                                                                const int8_t* __restrict__ pattern,
                                                                const double* __restrict__ bin_cs, int f_base,
                                                                uint8_t* __restrict__ out_des) {
  __shared__ uint32_t patch[kThreads / 64][kPatch * kPatchWords];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = blockIdx.y;
  const int k = blockIdx.x * (kThreads / 64) + wave;
  if (k >= kp_n[f_base + f]) return;  // wave-uniform; no block barriers below
  const size_t slot = (size_t)(f_base + f) * n_features + k;
  const uint32_t pp = kp_pos[slot];
  const int x = (int)(pp & 0xffffu), y = (int)(pp >> 16);
  const uint8_t* I = frames + (size_t)f * H * W;
  // rows y-15 .. y+15, bytes from bx = (x-15) & ~3 (x >= edge >= 16); the last word may
  // run up to 3 bytes past the row end, into the next row (y + 15 < H - 1)
  const int bx = (x - 15) & ~3, ofs = (x - 15) - bx;
  uint32_t* Pw = patch[wave];
  for (int i = lane; i < kPatch * kPatchWords; i += 64) {
    const int r = i / kPatchWords, c = i - r * kPatchWords;
    const uint8_t* src = I + (size_t)(y - 15 + r) * W + bx + 4 * c;
    uint32_t v;
    if ((W & 3) == 0) {
      v = *reinterpret_cast<const uint32_t*>(src);
    } else {
      v = 0;
      for (int b = 0; b < 4; ++b)
        if (bx + 4 * c + b < W) v |= (uint32_t)src[b] << (8 * b);
    }
    Pw[i] = v;
  }
  __builtin_amdgcn_wave_barrier();  // one wave writes and reads its slice: in order, no block barrier
  const uint8_t* P = reinterpret_cast<const uint8_t*>(Pw);
  int m10 = 0, m01 = 0;
  for (int i = lane; i < 31 * 31; i += 64) {
    const int dy = i / 31 - 15, dx = i % 31 - 15;
    if (dx * dx + dy * dy <= 225) {
      const int v = patch_at(P, ofs, dx, dy);
      m10 += dx * v;
      m01 += dy * v;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    m10 += __shfl_xor(m10, o);
    m01 += __shfl_xor(m01, o);
  }
  int bin = 0;
  if (m10 != 0 || m01 != 0) {
    int b = (int)floor(atan2((double)m01, (double)m10) / 0.19634954084936207);
    b &= 31;
    const int b1 = (b + 1) & 31;
    const double ck = (double)m01 * bin_cs[2 * b] - (double)m10 * bin_cs[2 * b + 1];
    const double ck1 = (double)m01 * bin_cs[2 * b1] - (double)m10 * bin_cs[2 * b1 + 1];
    bin = ck < 0 ? ((b + 31) & 31) : (ck1 >= 0 ? b1 : b);
  }
  const int8_t* pt = pattern + (size_t)bin * 512 * 2;
  uint8_t* d = out_des + slot * 32;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int pi = 64 * r + lane;
    const int p = smooth5_patch(P, ofs, pt[4 * pi], pt[4 * pi + 1]);
    const int q = smooth5_patch(P, ofs, pt[4 * pi + 2], pt[4 * pi + 3]);
    const unsigned long long m = __ballot(p < q);
    if (lane == 0) {
#pragma unroll
      for (int b = 0; b < 8; ++b) d[8 * r + b] = (uint8_t)(m >> (8 * b));
    }
  }
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_orb_detect(kcmc_ctx* ctx, const uint8_t* frames, int n_frames, int H, int W, int threshold,
                               int n_features, double harris_k, int edge, const int8_t* pattern, const double* bin_cs,
                               double* out_kp, uint8_t* out_des, int32_t* out_count, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_orb_detect: ctx is NULL");
  if (n_frames < 0 || H < 0 || W < 0 || n_features < 0) return fail(KCMC_EINVAL, "kcmc_orb_detect: negative size");
  if (n_frames == 0) return KCMC_OK;
  if (!frames || !pattern || !bin_cs || !out_kp || !out_des || !out_count)
    return fail(KCMC_EINVAL, "kcmc_orb_detect: NULL pointer");
  if (edge < 16) return fail(KCMC_EINVAL, "kcmc_orb_detect: edge must be >= 16 (orientation disc + BRIEF patch)");
  if (H > 65535 || W > 65535) return fail(KCMC_EUNSUPPORTED, "kcmc_orb_detect: H, W must be < 65536");
  if (threshold < 0 || threshold > 255) return fail(KCMC_EINVAL, "kcmc_orb_detect: threshold must be in [0, 255]");
  hipStream_t s = (hipStream_t)stream;
  KCMC_TRY(hip_check(hipMemsetAsync(out_count, 0, (size_t)n_frames * sizeof(int32_t), s), "hipMemsetAsync"));
  if (n_features == 0 || H < 2 * edge + 1 || W < 2 * edge + 1) return KCMC_OK;
  const int ntx = ceil_div(W, kTW), nty = ceil_div(H, kTH), ntiles = ntx * nty;
  // frames are processed in batches so that the candidate slots stay a bounded workspace
  const size_t slots = (size_t)ntiles * kSlots;
  const size_t per_frame = 2 * slots * (sizeof(uint64_t) + sizeof(uint32_t)) + (size_t)ntiles * 2 * sizeof(int32_t) + 4;
  int batch = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_frames, ((size_t)1 << 30) / per_frame));
  batch = std::min(batch, 65535);
  void* ws = nullptr;
  KCMC_TRY(workspace_alloc(ctx, &ws, per_frame * batch + (size_t)n_frames * n_features * sizeof(uint32_t) + 64, s));
  uint64_t* ckey = static_cast<uint64_t*>(ws);
  uint64_t* lkey = ckey + (size_t)batch * slots;
  uint32_t* cpos = reinterpret_cast<uint32_t*>(lkey + (size_t)batch * slots);
  uint32_t* lpos = cpos + (size_t)batch * slots;
  int32_t* ccnt = reinterpret_cast<int32_t*>(lpos + (size_t)batch * slots);
  int32_t* toff = ccnt + (size_t)batch * ntiles;
  int32_t* ctot = toff + (size_t)batch * ntiles;
  uint32_t* kpos = reinterpret_cast<uint32_t*>(ctot + batch);
  int rc = KCMC_OK;
  for (int f0 = 0; f0 < n_frames && rc == KCMC_OK; f0 += batch) {
    const int nb = std::min(batch, n_frames - f0);
    const uint8_t* fr = frames + (size_t)f0 * H * W;
    hipLaunchKernelGGL(orb_candidates_kernel, dim3(ntx, ceil_div(nty, kSub), nb), dim3(kThreads), 0, s, fr, H, W, threshold, harris_k,
                       edge, ckey, cpos, ccnt);
    hipLaunchKernelGGL(orb_offsets_kernel, dim3(nb), dim3(kThreads), 0, s, ccnt, ntiles, toff, ctot);
    hipLaunchKernelGGL(orb_gather_kernel, dim3(ceil_div(ntiles, 4 * 8), nb), dim3(kThreads), 0, s, ckey, cpos, ccnt,
                       toff, ntiles, lkey, lpos);
    hipLaunchKernelGGL(orb_select_kernel, dim3(nb), dim3(kThreads), 0, s, lkey, lpos, ctot, ntiles, n_features, out_kp,
                       kpos, out_count, f0);
    hipLaunchKernelGGL(orb_describe_kernel, dim3(ceil_div(n_features, kThreads / 64), nb), dim3(kThreads), 0, s, fr, H,
                       W, kpos, out_count, n_features, pattern, bin_cs, f0, out_des);
    rc = launch_check("orb kernels");
  }
  const int rc2 = workspace_free(ctx, ws, s);
  return rc != KCMC_OK ? rc : rc2;
}
