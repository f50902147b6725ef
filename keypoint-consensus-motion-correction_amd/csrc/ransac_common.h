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
// The same for a sequential fp64 sum Sd of the q (the model scorers' phase A): numpy's S is
// within (N + 3) 2^-53 S of the exact sum of the q, Sd within (N - 1) 2^-53 (2x margin); the
// range excludes every S == 0 (skimage's early exit) and the under / overflowing sums.
__device__ __forceinline__ double sd_eps(int N) { return (double)(2 * N + 8) * 0x1p-52; }
__device__ __forceinline__ bool sd_certain(double Sd) { return Sd >= 1e-290 && Sd <= 1e290; }

// ---------------------------------------------------------------- phase A in fp32
// The rigid scorer decides phase A in fp32 (round 6; fp64 VALU was 65 % of the scorers'
// instructions): a trial's map (X, Y) = a x + b y + t is rounded to fp32 and
// every point's residual e = (X - u, Y - v) and q = ex^2 + ey^2 are computed in fp32 from
// fp32 copies of the points centred on the frame's bounding boxes (x' = x - c_x, ...; the
// map's translation becomes t' = a c_x + b c_y + t - c_u, in fp64).  With
// M' = |a_x| h_x + |b_x| h_y + |t'_x| + h_u (h = the boxes' half extents, likewise for Y)
// and F = the same with the uncentred maxima, every |e32 - e| <= be = 7.01 2^-24 M' +
// 2^-49 F (the roundings of the inputs, of the map and of the three fp32 operations, plus
// the fp64 ones of the centring and of the reference's own e), so near q = tq
//   |q32 - q| <= B = 2 be sqrt(8 tq) + 2 be^2 + 8.5 2^-24 tq    (used with a 1.25 margin),
// and whenever B <= tq / 4: q32 < tq - B is an inlier, q32 > tq + B an outlier, for certain
// (far from tq the bound is relatively smaller still); points in between are counted as
// undecided, and a trial whose count the undecided points could lift to the best certain
// count is counted again in fp64 by a whole wave (phase A2).  S = sum r^2 is bracketed by
//   |S - S32| <= 2 be sqrt(2 N S') + 2 N be^2 + ((N + 2.1) 2^-24 + (N + 3) 2^-53) S'
// (Cauchy-Schwarz over the points; S' bounds the sum of the q32 from the fp32 sum S32).
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Mag {  // the frame's bounding boxes: centres, half extents, max magnitudes
  double cx, cy, cu, cv;  // (x, y): frame points; (u, v): template points
  double hx, hy, hu, hv;
  double X, Y, U, V;
};

struct Lin32 {
  f32x2 a, b, t;  // (X - u, Y - v) = a x' + b y' + t - u' in centred coordinates
  float lo, hi;   // certain inlier: q32 < lo; certain outlier: q32 > hi
  double be;
};

__device__ __forceinline__ bool lin32_make(double ax, double bx, double tx, double ay, double by, double ty,
                                           const Mag& mg, double tq, Lin32& L) {
  const double tpx = ax * mg.cx + bx * mg.cy + tx - mg.cu;
  const double tpy = ay * mg.cx + by * mg.cy + ty - mg.cv;
  const double Mx = fabs(ax) * mg.hx + fabs(bx) * mg.hy + fabs(tpx) + mg.hu;
  const double My = fabs(ay) * mg.hx + fabs(by) * mg.hy + fabs(tpy) + mg.hv;
  const double Fx = fabs(ax) * mg.X + fabs(bx) * mg.Y + fabs(tx) + mg.U;
  const double Fy = fabs(ay) * mg.X + fabs(by) * mg.Y + fabs(ty) + mg.V;
  const double be = 7.01 * 0x1p-24 * fmax(Mx, My) + 0x1p-49 * fmax(Fx, Fy);
  const double B = 1.25 * (2.0 * be * sqrt(8.0 * tq) + 2.0 * be * be + 8.5 * 0x1p-24 * tq);
  if (!(B <= 0.25 * tq) || !(tq < 1e30)) return false;  // NaN / huge maps and coordinates: fp64
  L.a = f32x2{(float)ax, (float)ay};
  L.b = f32x2{(float)bx, (float)by};
  L.t = f32x2{(float)tpx, (float)tpy};
  float lo = (float)(tq - B), hi = (float)(tq + B);
  // directed to the safe side (both positive: tq - B >= 3 tq / 4 > 0): one ulp down / up
  if ((double)lo > tq - B) lo = __int_as_float(__float_as_int(lo) - 1);
  if ((double)hi < tq + B) hi = __int_as_float(__float_as_int(hi) + 1);
  L.lo = lo;
  L.hi = hi;
  L.be = be;
  return true;
}

// The centred fp32 copy of point (x, y) -> (u, v).
__device__ __forceinline__ float4 centred32(double x, double y, double u, double v, const Mag& mg) {
  return make_float4((float)(x - mg.cx), (float)(y - mg.cy), (float)(u - mg.cu), (float)(v - mg.cv));
}

// Phase A of one trial in fp32 over the centred points (x', y', u', v') as float4 in LDS:
// returns S32, adds the certain inliers to clo and the certain-or-undecided ones to chi.
// Two points per iteration, so the reads of a pair are in flight together.
__device__ __forceinline__ float score32(const float4* __restrict__ pk, int N, const Lin32& L, int& clo, int& chi) {
  float S = 0.f;
  auto one = [&](const float4 p) {
    f32x2 e = L.t - f32x2{p.z, p.w};
    e = __builtin_elementwise_fma(L.b, f32x2{p.y, p.y}, e);
    e = __builtin_elementwise_fma(L.a, f32x2{p.x, p.x}, e);
    const float q = __builtin_fmaf(e.x, e.x, e.y * e.y);
    S += q;
    clo += q < L.lo ? 1 : 0;
    chi += q <= L.hi ? 1 : 0;
  };
  int k = 0;
  for (; k + 2 <= N; k += 2) {
    const float4 a = pk[k], b = pk[k + 1];
    one(a);
    one(b);
  }
  if (k < N) one(pk[k]);
  return S;
}

// [lo, hi] around numpy's S of a trial scored by score32 (the bound above, 1e-9 margins).
__device__ __forceinline__ void s32_bracket(float S32, int N, double be, double& lo, double& hi) {
  const double S = (double)S32;
  const double Sp = S * (1.0 + 1.01 * N * 0x1p-24);
  const double E = 2.0 * be * sqrt(2.02 * N * Sp) + 2.0 * N * be * be + ((N + 2.1) * 0x1p-24 + (N + 3) * 0x1p-53) * Sp;
  lo = (S - E) * (1.0 - 1e-9);
  hi = (S + E) * (1.0 + 1e-9);
}

// The fp64 phase A's bracket (s32_eps) in the same form.
__device__ __forceinline__ void s64_bracket(float S32, int N, double& lo, double& hi) {
  const double eps = s32_eps(N);
  lo = (double)S32 * (1.0 - eps);
  hi = (double)S32 * (1.0 + eps);
}

// The bracket of a wave's fp64 sum Sd of the q (phase A2): numpy's S is within
// (N + 3) 2^-53 S of the sum of the q, any summation order within (N - 1) 2^-53 (2x margin).
__device__ __forceinline__ void sd_bracket(double Sd, int N, double& lo, double& hi) {
  const double eps = (double)(2 * N + 8) * 0x1p-52;
  lo = Sd * (1.0 - eps);
  hi = Sd * (1.0 + eps);
}

// Phase A's per-trial record in the tC array: the certain inlier count and the undecided
// points (cnt | und << 16, counts <= kMaxN < 2^16), -1 for a trial without a model.
__device__ __forceinline__ int pack_cnt(int cnt, int und) { return cnt | (und << 16); }
__device__ __forceinline__ int cnt_of(int v) { return v < 0 ? v : (v & 0xffff); }
__device__ __forceinline__ int und_of(int v) { return v < 0 ? 0 : (v >> 16); }

__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// The boxes' centres, half extents and magnitudes from their bounds (lo, hi) per coordinate.
__device__ __forceinline__ Mag mag_of(const double (&L)[4], const double (&Hh)[4]) {
  double c[4], h[4], m[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool fin = fabs(L[i]) < INFINITY && fabs(Hh[i]) < INFINITY;
    c[i] = fin ? 0.5 * L[i] + 0.5 * Hh[i] : 0.0;
    h[i] = fin ? fmax(Hh[i] - c[i], c[i] - L[i]) * (1.0 + 0x1p-50) : INFINITY;  // >= every |x - c|
    m[i] = fmax(fabs(L[i]), fabs(Hh[i]));
  }
  Mag out;
  out.cx = c[0]; out.cy = c[1]; out.cu = c[2]; out.cv = c[3];
  out.hx = h[0]; out.hy = h[1]; out.hu = h[2]; out.hv = h[3];
  out.X = m[0]; out.Y = m[1]; out.U = m[2]; out.V = m[3];
  return out;
}

// One point's contribution to the bounds (a NaN or infinite coordinate makes them infinite).
__device__ __forceinline__ void mag_add(const double (&c)[4], double (&lo)[4], double (&hi)[4], bool& bad) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bad |= !(fabs(c[i]) < INFINITY);
    lo[i] = fmin(lo[i], c[i]);
    hi[i] = fmax(hi[i], c[i]);
  }
}

// The wave's bounds in every lane (min / max: exact in any order; a lane that saw a NaN or
// infinite coordinate contributes infinite bounds).
__device__ __forceinline__ void wave_bounds(double (&lo)[4], double (&hi)[4], bool bad) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (bad) {
      lo[i] = -INFINITY;
      hi[i] = INFINITY;
    }
    for (int o = 32; o > 0; o >>= 1) {
      lo[i] = fmin(lo[i], __shfl_xor(lo[i], o));
      hi[i] = fmax(hi[i], __shfl_xor(hi[i], o));
    }
  }
}

// The frame's bounding boxes for lin32_make: workgroup min / max over the staged points.
// A NaN or infinite coordinate makes the half extents infinite (every trial then runs the
// fp64 phase A).
// The result goes to the shared `out` (read per trial, not held in registers).
__device__ inline void frame_mag(const double* sx, const double* sy, const double* dx, const double* dy, int N,
                                 double* red, Mag& out) {
  double lo[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, hi[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  bool bad = false;
  for (int k = threadIdx.x; k < N; k += kThreads) {
    const double c[4] = {sx[k], sy[k], dx[k], dy[k]};
    mag_add(c, lo, hi, bad);
  }
  wave_bounds(lo, hi, bad);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      red[8 * wave + i] = lo[i];
      red[8 * wave + 4 + i] = hi[i];
    }
  __syncthreads();
  double L[4], Hh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    L[i] = red[i];
    Hh[i] = red[4 + i];
    for (int w = 1; w < kThreads / 64; ++w) {
      L[i] = fmin(L[i], red[8 * w + i]);
      Hh[i] = fmax(Hh[i], red[8 * w + 4 + i]);
    }
  }
  if (threadIdx.x == 0) out = mag_of(L, Hh);
  __syncthreads();  // out is visible, red is free
}

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
