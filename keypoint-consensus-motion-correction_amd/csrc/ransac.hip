// K2: batched rigid RANSAC with scikit-image 0.18.3 semantics.
//
// Reference: VA:288-323 (_compute_euclidean_affine) ->
//   skimage.measure.ransac((kp_query, kp_template), EuclideanTransform, min_samples=2,
//   residual_threshold=2, max_trials=1000, random_state=42)   (fit.py:621-881)
//
// One workgroup (4 waves) per frame.  The frame's N point pairs are staged in LDS
// (structure of arrays, read as broadcasts); each thread scores whole hypotheses:
//   model      closed-form 2-point rigid Umeyama (the rotation maximising tr(R^T A),
//              A = sum dst_d src_d^T; identical to skimage's SVD branch up to
//              rounding; A == 0 -> NaN model, never selected)
//   residual   r_k = sqrt(dx^2 + dy^2), x' = fma(y, -s, x*c) + tx (the order OpenBLAS
//              dgemm uses for skimage's [x y 1] @ M^T), inlier iff r_k < threshold
//   score      S = sum r_k^2 in numpy's pairwise-summation order (8 accumulators,
//              blocks of 128), so that hypotheses tie-break exactly like np.sum
// Selection: max inliers, then min S, then earliest trial (skimage's strict
// comparisons); skimage's early exit (best S <= 0) is emulated sequentially in the
// rare frames where some S == 0.  The hypothesis (sample pair) of trial t is the
// t-th RandomState(seed).choice(N, 2, replace=False), precomputed on the host per N
// (kcmc_ransac_prepare) -- it depends on N only because every frame reseeds.
// Refit: rigid Umeyama over the best inlier set (wave 0 alone for N <= 128, workgroup
// reductions above; the same sums in the same order either way).
#include <cfloat>
#include <cmath>

#include "kcmc_internal.h"
#include "ransac_common.h"

namespace kcmc {
namespace {

using namespace ransac_common;

struct Model {
  double c, s, tx, ty;
  bool ok;
};

// Closed-form rigid fit of two correspondences (skimage _umeyama, estimate_scale=False).
__device__ __forceinline__ Model fit2(double sx0, double sy0, double sx1, double sy1, double dx0, double dy0,
                                      double dx1, double dy1) {
  Model m;
  const double ms0 = (sx0 + sx1) / 2.0, ms1 = (sy0 + sy1) / 2.0;
  const double md0 = (dx0 + dx1) / 2.0, md1 = (dy0 + dy1) / 2.0;
  const double a0 = sx0 - ms0, a1 = sy0 - ms1, b0 = sx1 - ms0, b1 = sy1 - ms1;
  const double p0 = dx0 - md0, p1 = dy0 - md1, q0 = dx1 - md0, q1 = dy1 - md1;
  const double a00 = p0 * a0 + q0 * b0;
  const double a01 = p0 * a1 + q0 * b1;
  const double a10 = p1 * a0 + q1 * b0;
  const double a11 = p1 * a1 + q1 * b1;
  const double a = a00 + a11, b = a10 - a01;
  m.ok = !(a == 0.0 && b == 0.0);
  const double hn = sqrt(a * a + b * b);
  m.c = a / hn;
  m.s = b / hn;
  m.tx = md0 - (m.c * ms0 - m.s * ms1);
  m.ty = md1 - (m.s * ms0 + m.c * ms1);
  return m;
}

struct Pts {
  const double* sx;
  const double* sy;
  const double* dx;
  const double* dy;
};

__device__ __forceinline__ double resid2(const Model& m, const Pts& P, int k, double thresh, int& cnt) {
  const double x = P.sx[k], y = P.sy[k];
  const double xp = fma(y, -m.s, x * m.c) + m.tx;
  const double yp = fma(y, m.c, x * m.s) + m.ty;
  const double ex = xp - P.dx[k], ey = yp - P.dy[k];
  const double r = sqrt_resid(ex * ex + ey * ey);
  cnt += (r < thresh) ? 1 : 0;
  return r * r;
}

// numpy pairwise_sum over residual^2 of points [start, start+n) for n <= 128:
// n < 8 sequential, else 8 strided accumulators + sequential remainder.
__device__ __forceinline__ double pw_leaf(const Model& m, const Pts& P, int start, int n, double thresh, int& cnt) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += resid2(m, P, start + i, thresh, cnt);
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = resid2(m, P, start + j, thresh, cnt);
  int i = 8;
  const int nfull = n - (n % 8);
  for (; i < nfull; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += resid2(m, P, start + i + j, thresh, cnt);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += resid2(m, P, start + i, thresh, cnt);
  return res;
}

// Phase A of the scoring (see the kernel): the inlier count through the squared
// distance (r < thresh <=> q < tq, tq = the smallest double whose correctly rounded root
// is >= thresh; the q of every point is computed exactly as resid2 computes it) and an
// fp32 estimate of S = sum r_k^2: sum_k (float)q_k in sequence.  r_k^2 = q_k (1 + d),
// |d| <= 3 2^-53, numpy's pairwise sum adds <= N 2^-53 and the fp32 sum of N
// conversions <= (N + 1) 2^-24, so for S32 >= 1e-30 (no fp32 underflow matters)
// |S - S32| <= (N + 2) 2^-23 S32, used with a 2x margin.
__device__ __forceinline__ float score_fast(const Model& m, const Pts& P, int N, double tq, int& cnt) {
  float S = 0.f;
  for (int k = 0; k < N; ++k) {
    const double x = P.sx[k], y = P.sy[k];
    const double xp = fma(y, -m.s, x * m.c) + m.tx;
    const double yp = fma(y, m.c, x * m.s) + m.ty;
    const double ex = xp - P.dx[k], ey = yp - P.dy[k];
    const double q = ex * ex + ey * ey;
    cnt += (q < tq) ? 1 : 0;
    S += (float)q;
  }
  return S;
}

// For N > 128 the numpy pairwise order comes from the per-frame split Plan
// (ransac_common.h); invalid trials (NaN S, or 0 inliers with S = inf) never win.
// LARGE = false handles frames with N <= 128 (one pairwise leaf, fully in registers)
// and the NaN frames; LARGE = true handles 128 < N <= kMaxN through the split plan.
template <bool LARGE>
__device__ __forceinline__ void ransac_rigid_frame(
    int f, const double* __restrict__ src, const double* __restrict__ dst, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_off, int src_stride, const uint32_t* __restrict__ hyp,
    const int32_t* __restrict__ hyp_off, int hyp_off_len,
    int T, double thresh, double tq, double rate, int n_skip, double* __restrict__ out_params,
    uint8_t* __restrict__ out_inl, int32_t* __restrict__ out_nin, int32_t* __restrict__ out_best) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ double red[kThreads / 64 * 8];
  __shared__ int s_cnt[kThreads / 64];
  __shared__ double s_min[kThreads / 64];
  __shared__ int s_best[kThreads / 64 * 2];
  __shared__ double s_bestS[kThreads / 64];
  __shared__ int s_any_zero;
  __shared__ int s_final_t;
  __shared__ Plan s_plan;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int p0 = pt_off[f];
  const int N = pt_off[f + 1] - p0;

  const bool skip_frame = N < n_skip || N < 3 || N > kMaxN;
  const int hoff = (!skip_frame && N < hyp_off_len) ? hyp_off[N] : -1;
  const bool nan_frame = skip_frame || hoff < 0;
  if (LARGE != (!nan_frame && N > 128)) return;  // the other launch owns this frame
  if (nan_frame) {
    if (tid < 6) out_params[6 * (size_t)f + tid] = NAN;
    for (int k = tid; k < N; k += kThreads) out_inl[p0 + k] = 0;
    if (tid == 0) {
      out_nin[f] = skip_frame ? 0 : -1;  // -1: no hypothesis table was prepared for N
      out_best[f] = -1;
    }
    return;
  }
  const uint32_t* H = hyp + hoff;

  // LDS: sx, sy, dx, dy [N] f64 | the points as (x, y, u, v) [N] f32x4 | trial S (low bound)
  //      [T] f64 | trial S high bound [T] f64 | [LARGE: stack [kMaxStack][256] f64]
  //      | per-wave leaf values [4][128] f64 | trial count [T] i32 | inlier flags [N] u8
  double* sx = smem;
  double* sy = sx + N;
  double* dxs = sy + N;
  double* dys = dxs + N;
  float4* pk32 = reinterpret_cast<float4*>(dys + N);  // 16-byte aligned: 4 N doubles before it
  double* tS = reinterpret_cast<double*>(pk32 + N);
  double* tSh = tS + T;
  double* stk = tSh + T;
  double* wvals = stk + (LARGE ? kMaxStack * kThreads : 0);
  int* tC = reinterpret_cast<int*>(wvals + kThreads / 64 * 128);
  uint8_t* inl = reinterpret_cast<uint8_t*>(tC + T);
  if (LARGE && tid == 0) {
    s_plan.n = 0;
    plan_gen<kPwDepth>(s_plan, 0, N);
  }

  auto gather = [&](int k, double (&c)[4]) {
    size_t si, di;
    if (pt_idx) {
      const int q = pt_idx[p0 + k];
      si = (size_t)f * src_stride + q;
      di = (size_t)q;
    } else {
      si = di = (size_t)(p0 + k);
    }
    c[0] = src[2 * si];
    c[1] = src[2 * si + 1];
    c[2] = dst[2 * di];
    c[3] = dst[2 * di + 1];
  };
  if (tid == 0) s_any_zero = 0;
  __shared__ Mag mg;
  if (!LARGE) {
    // N <= 128: wave 0 stages every point (k = lane, lane + 64), takes the frame's boxes by
    // wave reductions (min / max: the same bounds in any order) and writes the fp32 copies,
    // behind one barrier (the workgroup form takes five)
    if (wave == 0) {
      double c[2][4], lo[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, hi[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      bool bad = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < N) {
          gather(k, c[h]);
          mag_add(c[h], lo, hi, bad);
        }
      }
      wave_bounds(lo, hi, bad);
      const Mag m = mag_of(lo, hi);
      if (lane == 0) mg = m;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < N) {
          sx[k] = c[h][0];
          sy[k] = c[h][1];
          dxs[k] = c[h][2];
          dys[k] = c[h][3];
          pk32[k] = centred32(c[h][0], c[h][1], c[h][2], c[h][3], m);
        }
      }
    }
    __syncthreads();
  } else {
    for (int k = tid; k < N; k += kThreads) {
      double c[4];
      gather(k, c);
      sx[k] = c[0];
      sy[k] = c[1];
      dxs[k] = c[2];
      dys[k] = c[3];
    }
    __syncthreads();
    frame_mag(sx, sy, dxs, dys, N, red, mg);
    for (int k = tid; k < N; k += kThreads) pk32[k] = centred32(sx[k], sy[k], dxs[k], dys[k], mg);
    __syncthreads();
  }

  const Pts P{sx, sy, dxs, dys};

  // ---- phase A: every trial's inlier count and a bracket [tS, tSh] of its S.  In fp32
  // (ransac_common.h score32: certain inliers, outliers and the undecided points between
  // them; a trial whose map or frame is too large for the fp32 bound runs the fp64 form,
  // score_fast).  A trial whose undecided points could lift it to the best certain count
  // is scored again in fp64 (phase A2), so the best count is exact.  Then only trials at
  // that count whose bracket reaches the smallest upper bound need the exact S (phase B,
  // one whole wave per candidate).  Frames the brackets cannot decide -- no trial with
  // inliers, a bracket outside [1e-30, 1e30] (so also every S == 0, skimage's early exit),
  // or a NaN tq -- score every trial exactly (the original single-phase loop).
  const bool fast = tq == tq;  // NaN: exact scoring only (threshold outside the fast range)
  int mcount = -1, flag = fast ? 0 : 1;
  if (fast) {
    int mlo = -1;
    bool deferred = false;  // trials the fp32 bound cannot take: the fp64 loop below
    for (int t = tid; t < T; t += kThreads) {
      const uint32_t pr = H[t];
      const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
      const Model m = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
      int v = -1;
      double slo = NAN, shi = NAN;
      Lin32 L;
      if (m.ok && lin32_make(m.c, -m.s, m.tx, m.s, m.c, m.ty, mg, tq, L)) {
        int clo = 0, chi = 0;
        const float S32 = score32(pk32, N, L, clo, chi);
        s32_bracket(S32, N, L.be, slo, shi);
        v = pack_cnt(clo, chi - clo);
        if (!(slo >= 1e-30 && shi <= 1e30)) flag = 1;
      } else if (m.ok) {
        v = INT_MIN;
        deferred = true;
      }
      tC[t] = v;
      tS[t] = slo;
      tSh[t] = shi;
      mlo = max(mlo, cnt_of(v));
    }
    if (deferred) {
      for (int t = tid; t < T; t += kThreads) {
        if (tC[t] != INT_MIN) continue;
        const uint32_t pr = H[t];
        const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
        const Model m = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
        int cnt = 0;
        const float S32 = score_fast(m, P, N, tq, cnt);
        double slo, shi;
        s64_bracket(S32, N, slo, shi);
        if (!(slo >= 1e-30 && shi <= 1e30)) flag = 1;
        tC[t] = cnt;
        tS[t] = slo;
        tSh[t] = shi;
        mlo = max(mlo, cnt);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      mlo = max(mlo, __shfl_xor(mlo, o));
      flag |= __shfl_xor(flag, o);
    }
    if (lane == 0) s_cnt[wave] = (mlo + 1) | (flag << 30);  // counts <= kMaxN
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
      const int v = s_cnt[w];
      flag |= v >> 30;
      mlo = max(mlo, (v & 0x3fffffff) - 1);
    }
    __syncthreads();  // s_cnt is reused
    // phase A2: the exact count of every trial the undecided points could lift to mlo, each
    // by a whole wave (the points over the lanes, fp64 as score_fast computes them)
    for (int t0 = wave * 64; t0 < T; t0 += kThreads) {
      const int t = t0 + lane;
      uint64_t need = __ballot(!flag && t < T && und_of(tC[t]) > 0 && cnt_of(tC[t]) + und_of(tC[t]) >= mlo);
      while (need) {
        const int tc = t0 + __builtin_ctzll(need);
        need &= need - 1;
        const uint32_t pr = H[tc];
        const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
        const Model m = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
        int c = 0;
        double sq = 0.0;
        for (int k = lane; k < N; k += 64) {
          const double x = sx[k], y = sy[k];
          const double xp = fma(y, -m.s, x * m.c) + m.tx;
          const double yp = fma(y, m.c, x * m.s) + m.ty;
          const double ex = xp - dxs[k], ey = yp - dys[k];
          const double q = ex * ex + ey * ey;
          c += (q < tq) ? 1 : 0;
          sq += q;
        }
        c = wave_sum_i(c);
        double slo, shi;
        sd_bracket(wave_sum(sq), N, slo, shi);
        if (!(slo >= 1e-30 && shi <= 1e30)) flag = 1;
        if (lane == 0) {
          tC[tc] = c;
          tS[tc] = slo;
          tSh[tc] = shi;
        }
      }
    }
    __syncthreads();  // the A2 results of the other waves' lanes
    for (int t = tid; t < T; t += kThreads) mcount = max(mcount, cnt_of(tC[t]));
  }
  for (int o = 32; o > 0; o >>= 1) {
    mcount = max(mcount, __shfl_xor(mcount, o));
    flag |= __shfl_xor(flag, o);
  }
  if (lane == 0) s_cnt[wave] = (mcount + 1) | (flag << 30);  // counts <= kMaxN
  __syncthreads();
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    const int v = s_cnt[w];
    flag |= v >> 30;
    mcount = max(mcount, (v & 0x3fffffff) - 1);
  }
  const bool exact = flag != 0 || mcount <= 0;

  int bc = -1, bt = INT_MAX;
  double bS = INFINITY;
  bool any_zero = false;
  if (exact) {
    for (int t = tid; t < T; t += kThreads) {
      const uint32_t pr = H[t];
      const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
      const Model m = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
      int cnt = 0;
      double S = NAN;
      if (m.ok) {
        if (!LARGE) {
          S = pw_leaf(m, P, 0, N, thresh, cnt);
        } else {
          int sp = 0;
          for (int l = 0; l < s_plan.n; ++l) {
            stk[sp++ * kThreads + tid] = pw_leaf(m, P, s_plan.start[l], s_plan.len[l], thresh, cnt);
            for (int c = s_plan.pops[l]; c > 0; --c) {
              const double b = stk[--sp * kThreads + tid];
              const double a = stk[(sp - 1) * kThreads + tid];
              stk[(sp - 1) * kThreads + tid] = a + b;
            }
          }
          S = stk[tid];
        }
      }
      tS[t] = S;
      tC[t] = cnt;
      const bool valid = !isnan(S) && (cnt > 0 || S < INFINITY);
      if (valid) {
        if (S <= 0.0) any_zero = true;
        if (better(cnt, S, t, bc, bS, bt)) {
          bc = cnt;
          bS = S;
          bt = t;
        }
      }
    }
  } else {
    double lm = INFINITY;
    for (int t = tid; t < T; t += kThreads)
      if (cnt_of(tC[t]) == mcount) lm = fmin(lm, tSh[t]);
    for (int o = 32; o > 0; o >>= 1) lm = fmin(lm, __shfl_xor(lm, o));
    if (lane == 0) s_min[wave] = lm;
    __syncthreads();
    const double minhi = fmin(fmin(s_min[0], s_min[1]), fmin(s_min[2], s_min[3]));
    double* vals = wvals + wave * 128;
    double* wstk = stk + wave * kMaxStack;  // LARGE: the wave's combine stack (uniform values)
    // phase B: this wave's candidate trials (t = t0 + lane), each scored by the whole wave
    for (int t0 = wave * 64; t0 < T; t0 += kThreads) {
      const int t = t0 + lane;
      uint64_t cand = __ballot(t < T && cnt_of(tC[t]) == mcount && tS[t] <= minhi);
      while (cand) {
        const int tc = t0 + __builtin_ctzll(cand);
        cand &= cand - 1;
        const uint32_t pr = H[tc];
        const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
        const Model m = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
        const double S = wave_pairwise<LARGE>(
            [&](int k) {
              int c = 0;
              return resid2(m, P, k, thresh, c);
            },
            N, s_plan, vals, wstk, lane);
        if (!isnan(S) && better(mcount, S, tc, bc, bS, bt)) {  // wave-uniform
          bc = mcount;
          bS = S;
          bt = tc;
        }
      }
    }
  }
  // workgroup argmax of (count, -S, -t)
  for (int o = 32; o > 0; o >>= 1) {
    const int oc = __shfl_xor(bc, o);
    const double oS = __shfl_xor(bS, o);
    const int ot = __shfl_xor(bt, o);
    if (better(oc, oS, ot, bc, bS, bt)) {
      bc = oc;
      bS = oS;
      bt = ot;
    }
  }
  if (lane == 0) {
    s_best[2 * wave] = bc;
    s_best[2 * wave + 1] = bt;
    s_bestS[wave] = bS;
  }
  if (any_zero) atomicOr(&s_any_zero, 1);
  __syncthreads();
  if (tid == 0) {
    int fc = -1, ft = INT_MAX;
    double fS = INFINITY;
    for (int w = 0; w < kThreads / 64; ++w)
      if (better(s_best[2 * w], s_bestS[w], s_best[2 * w + 1], fc, fS, ft)) {
        fc = s_best[2 * w];
        fS = s_bestS[w];
        ft = s_best[2 * w + 1];
      }
    if (s_any_zero) {
      // skimage stops as soon as the running best has S <= 0 (fit.py:862-869):
      // replay the trial sequence to find where it stopped.
      int c0 = 0, t0 = -1;
      double S0 = INFINITY;
      for (int t = 0; t < T; ++t) {
        const double S = tS[t];
        const int c = tC[t];
        if (isnan(S)) continue;
        if (c > c0 || (c == c0 && S < S0)) {
          c0 = c;
          S0 = S;
          t0 = t;
          if (S0 <= 0.0) break;
        }
      }
      ft = t0;
      fc = c0;
    }
    s_final_t = (ft == INT_MAX) ? -1 : ft;
  }
  __syncthreads();
  const int best_t = s_final_t;

  // inlier mask of the best hypothesis (same arithmetic as the scoring loop)
  int nin_local = 0;
  Model bm{0, 0, 0, 0, false};
  if (best_t >= 0) {
    const uint32_t pr = H[best_t];
    const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
    bm = fit2(sx[i], sy[i], sx[j], sy[j], dxs[i], dys[i], dxs[j], dys[j]);
  }
  for (int k = tid; k < N; k += kThreads) {
    int c = 0;
    if (bm.ok) resid2(bm, P, k, thresh, c);
    inl[k] = (uint8_t)c;
    out_inl[p0 + k] = (uint8_t)c;
    nin_local += c;
  }
  __syncthreads();
  // refit on the inliers (skimage fit.py:871-875 -> _umeyama over d[best_inliers])
  double n_in, ms0, ms1, md0, md1, a00 = 0, a01 = 0, a10 = 0, a11 = 0;
  if (!LARGE) {
    // N <= 128: wave 0 alone, with no barrier.  Lane l holds points l and l + 64, the
    // points threads l and l + 64 hold in the workgroup form below; each half goes through
    // the same butterfly as there, and the halves are added as block_sum adds its four wave
    // sums (0 + wave 0 + wave 1 + 0 + 0), so every sum is the same to the bit.
    if (wave != 0) return;
    const int k1 = lane + 64;
    const bool i0 = lane < N && inl[lane], i1 = k1 < N && inl[k1];
    auto half_sums = [&](double lo, double hi) {
      for (int o = 32; o > 0; o >>= 1) {
        lo += __shfl_xor(lo, o);
        hi += __shfl_xor(hi, o);
      }
      return (((0.0 + lo) + hi) + 0.0) + 0.0;
    };
    n_in = half_sums(i0 ? 1.0 : 0.0, i1 ? 1.0 : 0.0);
    ms0 = half_sums(i0 ? 0.0 + sx[lane] : 0.0, i1 ? 0.0 + sx[k1] : 0.0) / n_in;
    ms1 = half_sums(i0 ? 0.0 + sy[lane] : 0.0, i1 ? 0.0 + sy[k1] : 0.0) / n_in;
    md0 = half_sums(i0 ? 0.0 + dxs[lane] : 0.0, i1 ? 0.0 + dxs[k1] : 0.0) / n_in;
    md1 = half_sums(i0 ? 0.0 + dys[lane] : 0.0, i1 ? 0.0 + dys[k1] : 0.0) / n_in;
    double b[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = h ? k1 : lane;
      if (h ? i1 : i0) {
        const double u0 = sx[k] - ms0, u1 = sy[k] - ms1;
        const double v0 = dxs[k] - md0, v1 = dys[k] - md1;
        b[h][0] = 0.0 + v0 * u0;
        b[h][1] = 0.0 + v0 * u1;
        b[h][2] = 0.0 + v1 * u0;
        b[h][3] = 0.0 + v1 * u1;
      }
    }
    a00 = half_sums(b[0][0], b[1][0]);
    a01 = half_sums(b[0][1], b[1][1]);
    a10 = half_sums(b[0][2], b[1][2]);
    a11 = half_sums(b[0][3], b[1][3]);
  } else {
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0, cntd = 0;
    for (int k = tid; k < N; k += kThreads)
      if (inl[k]) {
        s0 += sx[k];
        s1 += sy[k];
        s2 += dxs[k];
        s3 += dys[k];
        cntd += 1.0;
      }
    n_in = block_sum(cntd, red);
    ms0 = block_sum(s0, red) / n_in;
    ms1 = block_sum(s1, red) / n_in;
    md0 = block_sum(s2, red) / n_in;
    md1 = block_sum(s3, red) / n_in;
    for (int k = tid; k < N; k += kThreads)
      if (inl[k]) {
        const double u0 = sx[k] - ms0, u1 = sy[k] - ms1;
        const double v0 = dxs[k] - md0, v1 = dys[k] - md1;
        a00 += v0 * u0;
        a01 += v0 * u1;
        a10 += v1 * u0;
        a11 += v1 * u1;
      }
    a00 = block_sum(a00, red);
    a01 = block_sum(a01, red);
    a10 = block_sum(a10, red);
    a11 = block_sum(a11, red);
  }
  if (tid == 0) {
    double* o = out_params + 6 * (size_t)f;
    const double a = a00 + a11, b = a10 - a01;
    if (n_in > 0.0 && !(a == 0.0 && b == 0.0)) {
      const double hn = sqrt(a * a + b * b);
      const double c = a / hn, s = b / hn;
      o[0] = c;
      o[1] = -s;
      o[2] = (md0 - (c * ms0 - s * ms1)) * rate;
      o[3] = s;
      o[4] = c;
      o[5] = (md1 - (s * ms0 + c * ms1)) * rate;
    } else {
      for (int k = 0; k < 6; ++k) o[k] = NAN;
    }
    out_nin[f] = (int32_t)n_in;
    out_best[f] = best_t;
  }
  (void)nin_local;
}

// Workgroup g scores frames g, g + grid, ... (the product launches one workgroup per frame;
// narrower grids measured slower beside the warp).
template <bool LARGE>
__global__ __launch_bounds__(kThreads, 4) void ransac_rigid_kernel(
    int n_frames, const double* __restrict__ src, const double* __restrict__ dst, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_off, int src_stride, const uint32_t* __restrict__ hyp,
    const int32_t* __restrict__ hyp_off, int hyp_off_len,
    int T, double thresh, double tq, double rate, int n_skip, double* __restrict__ out_params,
    uint8_t* __restrict__ out_inl, int32_t* __restrict__ out_nin, int32_t* __restrict__ out_best) {
  for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
    ransac_rigid_frame<LARGE>(f, src, dst, pt_idx, pt_off, src_stride, hyp, hyp_off, hyp_off_len, T, thresh, tq, rate,
                              n_skip, out_params, out_inl, out_nin, out_best);
    __syncthreads();  // the frame's LDS is free for the next one
  }
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

static int ransac_rigid_impl(kcmc_ctx* ctx, const double* src, const double* dst, const int32_t* pt_idx,
                                 const int32_t* pt_off, int src_frame_stride, int n_frames, int max_n, int trials,
                                 double thresh, double rate, int n_skip, double* out_params, uint8_t* out_inliers,
                                 int32_t* out_n_inliers, int32_t* out_best_trial, int max_workgroups, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_ransac_rigid: ctx is NULL");
  if (n_frames < 0 || max_n < 0 || trials < 1) return fail(KCMC_EINVAL, "kcmc_ransac_rigid: bad sizes");
  if (n_frames == 0) return KCMC_OK;
  if (!pt_off || !out_params || !out_n_inliers || !out_best_trial || (max_n > 0 && (!src || !dst || !out_inliers)))
    return fail(KCMC_EINVAL, "kcmc_ransac_rigid: NULL pointer");
  if (max_n > kMaxN) return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_rigid: max_n > 4096 points per frame");
  if (pt_idx && src_frame_stride <= 0) return fail(KCMC_EINVAL, "kcmc_ransac_rigid: src_frame_stride must be > 0");
  const int need = max_n < 3 ? 3 : max_n;
  if (!ctx->hyp || ctx->hyp_trials != trials)
    return fail(KCMC_EINVAL, "kcmc_ransac_rigid: hypothesis tables not prepared for trials=" +
                                 std::to_string(trials) + " (call kcmc_ransac_prepare)");
  const int n_small = need < 128 ? need : 128;
  const size_t wvals = (size_t)kThreads / 64 * 128 * sizeof(double);
  // per point 4 f64 + one f32x4, per trial 2 f64 + one i32
  const size_t lds_small = (size_t)n_small * (4 * sizeof(double) + 16) + (size_t)trials * (2 * sizeof(double) + sizeof(int)) +
                           wvals + (size_t)n_small + 16;
  const size_t lds_large = (size_t)need * (4 * sizeof(double) + 16) + (size_t)trials * (2 * sizeof(double) + sizeof(int)) +
                           (size_t)kMaxStack * kThreads * sizeof(double) + wvals + (size_t)need + 16;
  const double tq = inlier_bound(thresh);
  if ((max_n > 128 ? lds_large : lds_small) > 150 * 1024)
    return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_rigid: max_n/trials exceed the LDS budget");
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)(max_workgroups > 0 && max_workgroups < n_frames ? max_workgroups : n_frames);
  hipLaunchKernelGGL(ransac_rigid_kernel<false>, dim3(grid), dim3(kThreads), lds_small, s, n_frames, src, dst, pt_idx,
                     pt_off, src_frame_stride, ctx->hyp, ctx->hyp_off, ctx->hyp_off_len, trials, thresh, tq, rate, n_skip,
                     out_params, out_inliers, out_n_inliers, out_best_trial);
  KCMC_TRY(launch_check("ransac_rigid_kernel<small>"));
  if (max_n > 128) {
    hipLaunchKernelGGL(ransac_rigid_kernel<true>, dim3(grid), dim3(kThreads), lds_large, s, n_frames, src, dst, pt_idx,
                       pt_off, src_frame_stride, ctx->hyp, ctx->hyp_off, ctx->hyp_off_len, trials, thresh, tq, rate, n_skip,
                       out_params, out_inliers, out_n_inliers, out_best_trial);
    KCMC_TRY(launch_check("ransac_rigid_kernel<large>"));
  }
  return KCMC_OK;
}

extern "C" int kcmc_ransac_rigid(kcmc_ctx* ctx, const double* src, const double* dst, const int32_t* pt_idx,
                                 const int32_t* pt_off, int src_frame_stride, int n_frames, int max_n, int trials,
                                 double thresh, double rate, int n_skip, double* out_params, uint8_t* out_inliers,
                                 int32_t* out_n_inliers, int32_t* out_best_trial, kcmc_stream_t stream) {
  return ransac_rigid_impl(ctx, src, dst, pt_idx, pt_off, src_frame_stride, n_frames, max_n, trials, thresh, rate, n_skip, out_params, out_inliers, out_n_inliers, out_best_trial, 0, stream);
}
