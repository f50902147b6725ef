// Model-independent pieces of the batched RANSAC kernels (ransac.hip: rigid,
// ransac_model.hip: affine / projective): launch shape, numpy's pairwise-summation
// split plan, skimage's selection order and workgroup / wave sums.
#pragma once

#include <climits>
#include <cmath>
#include <cstdint>

#include "kcmc_internal.h"

namespace kcmc {
namespace ransac_common {

constexpr int kThreads = 256;
constexpr int kMaxN = 4096;  // numpy's pairwise split tree has depth <= 6 for n <= 4096
constexpr int kPwDepth = 6;

// For n > 128 numpy's pairwise_sum recurses: pairwise(a, n) = pairwise(a, n2) +
// pairwise(a + n2, n - n2) with n2 = n/2 rounded down to a multiple of 8.  The split
// tree depends on N only, so one thread writes it once per frame as a post-order plan:
// leaves in order, each with the number of "pop b, pop a, push a+b" combines that
// follow it.  Every thread then evaluates its hypotheses with one copy of the leaf
// loop and a per-thread stack in LDS.
constexpr int kMaxLeaves = 128;
constexpr int kMaxStack = kPwDepth + 2;

struct Plan {
  int16_t start[kMaxLeaves];
  int16_t len[kMaxLeaves];
  int8_t pops[kMaxLeaves];
  int n;
};

template <int DEPTH>
__device__ __forceinline__ void plan_gen(Plan& p, int s, int n) {
  if (DEPTH == 0 || n <= 128) {
    p.start[p.n] = (int16_t)s;
    p.len[p.n] = (int16_t)n;
    p.pops[p.n] = 0;
    ++p.n;
    return;
  }
  if constexpr (DEPTH > 0) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    plan_gen<DEPTH - 1>(p, s, n2);
    plan_gen<DEPTH - 1>(p, s + n2, n - n2);
    ++p.pops[p.n - 1];
  }
}

// sqrt of a squared residual distance, the hot op of every scoring loop: the same
// rsq + Goldschmidt/Newton sequence (and so the same correctly rounded result) that
// the compiler emits for sqrt(double), without its denormal-range scaling and its
// zero/infinity selects (~7 of ~32 VALU per residual).  Identical to sqrt(d) for
// d == 0, d >= 2^-767 (|residual| >= 2^-383) and NaN; d = +inf (coordinates beyond
// 1e154) gives NaN instead of inf.  rsq of max(d, 2^-1000) keeps d == 0 finite:
// g = 0 * 2^500 = 0 and every correction term stays 0.
__device__ __forceinline__ double sqrt_resid(double d) {
  const double y = __builtin_amdgcn_rsq(fmax(d, 0x1p-1000));
  double g = d * y;
  double h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double e = fma(-g, g, d);
  g = fma(e, h, g);
  e = fma(-g, g, d);
  return fma(e, h, g);
}

// skimage's selection order (fit.py:851-861): (count desc, S asc, trial asc).
__device__ __forceinline__ bool better(int c, double S, int t, int bc, double bS, int bt) {
  if (c != bc) return c > bc;
  if (S != bS) return S < bS;
  return t < bt;
}

// tq = the smallest double whose correctly rounded square root is >= thresh, so that
// sqrt(q) < thresh <=> q < tq for every q (the root is monotone; NaN compares false
// either way): the scoring kernels' phase A counts inliers without the root.
// sqrt_resid is the correctly rounded root for q >= 2^-767, so thresholds whose tq falls
// below that (or non-finite / non-positive ones) return NaN: exact scoring only.
inline double inlier_bound(double thresh) {
  if (!(thresh > 0x1p-380 && thresh < 0x1p500)) return NAN;
  double q = thresh * thresh;
  while (std::sqrt(q) < thresh) q = std::nextafter(q, INFINITY);
  for (double p = std::nextafter(q, 0.0); std::sqrt(p) >= thresh; p = std::nextafter(q, 0.0)) q = p;
  return q;
}

// Phase B of the scoring kernels: numpy's pairwise leaf (8 strided accumulators for
// n >= 8, sequential below; n <= 128) over r2(start + k), evaluated by one whole wave:
// the lanes write the values to the wave's LDS row `vals`, lanes j < 8 run accumulator
// j's sequential sum, and every lane finishes the same combine and remainder
// (wave-uniform result, bit-identical to a one-thread pw_leaf).
template <class R2>
__device__ __forceinline__ double wave_leaf(R2 r2, int start, int n, double* vals, int lane) {
  for (int k = lane; k < n; k += 64) vals[k] = r2(start + k);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double res = 0.0;
  if (n < 8) {
    for (int i = 0; i < n; ++i) res += vals[i];
  } else {
    const int j = lane & 7;
    const int nfull = n - (n % 8);
    double r = vals[j];
    for (int i = j + 8; i < nfull; i += 8) r += vals[i];
    double rj[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) rj[q] = __shfl(r, q);
    res = ((rj[0] + rj[1]) + (rj[2] + rj[3])) + ((rj[4] + rj[5]) + (rj[6] + rj[7]));
    for (int i = nfull; i < n; ++i) res += vals[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // vals is rewritten by the next leaf
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return res;
}

// The exact S of one trial by one wave: a single leaf for N <= 128, else numpy's split
// plan with the combine stack in the wave's LDS slots `wstk` (uniform values).
template <bool LARGE, class R2>
__device__ __forceinline__ double wave_pairwise(R2 r2, int N, const Plan& plan, double* vals, double* wstk, int lane) {
  if (!LARGE) return wave_leaf(r2, 0, N, vals, lane);
  int sp = 0;
  for (int l = 0; l < plan.n; ++l) {
    wstk[sp++] = wave_leaf(r2, plan.start[l], plan.len[l], vals, lane);
    for (int c = plan.pops[l]; c > 0; --c) {
      const double b = wstk[--sp];
      const double a = wstk[sp - 1];
      wstk[sp - 1] = a + b;
    }
  }
  return wstk[0];
}

// Phase A's error bound (the kernels' comment): |S - S32| <= eps S32 for S32 in
// [1e-30, 1e30], with a 2x margin.
__device__ __forceinline__ double s32_eps(int N) { return (double)(N + 2) * 0x1p-22; }
__device__ __forceinline__ bool s32_certain(float S32) { return S32 >= 1e-30f && S32 <= 1e30f; }

__device__ inline double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  return s;
}

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace ransac_common
}  // namespace kcmc
