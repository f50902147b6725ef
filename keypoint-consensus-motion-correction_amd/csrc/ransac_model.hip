// K2 extension: batched affine / projective RANSAC with scikit-image 0.18.3 semantics.
//
// The reference fits EuclideanTransform only (VA:311, kernel in ransac.hip).  BASELINE
// configs 3-5 ask for affine and homography models; this file implements
//   skimage.measure.ransac((src, dst), AffineTransform,     min_samples=3, ...)
//   skimage.measure.ransac((src, dst), ProjectiveTransform, min_samples=4, ...)
// (fit.py:621-881; _geometric.py:18-69, 548-562, 596-703, 746-845) with the seeded
// hypothesis stream skimage draws: trial t uses the t-th
// RandomState(seed).choice(N, k, replace=False) = the first k entries of the t-th
// legacy MT19937 permutation of N (host tables per (k, N), kcmc_ransac_prepare_samples).
//
// ransac_model_score_kernel -- one workgroup per frame, the N point pairs in LDS, one
//   thread per hypothesis:
//   * minimal fit: affine = the exact 3-point solve (what skimage's total-least-squares
//     SVD returns for a non-degenerate triple); projective = the 8x8 DLT system in
//     Hartley-normalised coordinates with h22 = 1 (skimage's normalisation and scale),
//     Gaussian elimination with partial pivoting, de-normalised like skimage;
//   * skimage's degeneracy tests, where estimate() returns False and the trial is
//     skipped (fit.py:835-838): a sample with rms 0 (ZeroDivisionError), a singular
//     system, or np.isclose(V[-1,-1], 0) <=> 1/sqrt(1 + |h|^2) <= 1e-8 with h the model
//     in normalised coordinates;
//   * residuals as _apply_mat computes them ([x y 1] @ H^T in the dgemm operation
//     order used for the rigid model; w == 0 -> eps; divide), inlier iff r < threshold,
//     S = sum r^2 in numpy's pairwise order;
//   * selection (count desc, S asc, trial asc) with skimage's S <= 0 early exit, then
//     the winner's inlier mask and model.
// refit_frame (fused at the end of each scoring workgroup) -- one wave per frame: the final total-least-squares fit on
//   the inliers (fit.py:871-875 -> ProjectiveTransform.estimate): Hartley
//   normalisation, the last right singular vector of the 2N x 7 (affine) / 2N x 9
//   (projective) system A that skimage takes from np.linalg.svd -- by a Givens QR of A in
//   the wave and a one-sided Jacobi SVD of its triangle, in fp64 -- then
//   H = inv(N_dst) Hn N_src.  As in skimage, a refit with |v_last| <= 1e-8 keeps the
//   hypothesis model and rms == 0 gives NaN.
// Output params [F, 3, 3] (row-major), NaN where skimage returns no model, scaled for
// spatial downsampling as S H S^-1 with S = diag(rate, rate, 1) (for affine models
// exactly the reference's translation scaling, VA:320).
#include <cfloat>
#include <cmath>

#include "kcmc_internal.h"
#include "ransac_common.h"

namespace kcmc {
namespace {

using namespace ransac_common;

constexpr double kSqrt2 = 1.4142135623730951;  // math.sqrt(2)

struct HModel {
  double h[9];
  bool ok;
};

struct Pts {
  const double* sx;
  const double* sy;
  const double* dx;
  const double* dy;
};

// skimage _center_and_normalize_points for the K sample points: centroid = numpy's
// sequential axis-0 mean, rms = sqrt(pairwise_sum of the 2K squared deviations / K)
// (2K < 8: sequential; 2K == 8: numpy's 8-accumulator combine).  false: rms == 0.
template <int K>
__device__ __forceinline__ bool center_normalize(const double* px, const double* py, const int (&sel)[K], double& cx,
                                                 double& cy, double& nf) {
  double sx = 0.0, sy = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    sx += px[sel[i]];
    sy += py[sel[i]];
  }
  cx = sx / K;
  cy = sy / K;
  double dev[2 * K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const double ex = px[sel[i]] - cx, ey = py[sel[i]] - cy;
    dev[2 * i] = ex * ex;
    dev[2 * i + 1] = ey * ey;
  }
  double ss;
  if constexpr (2 * K < 8) {
    ss = 0.0;
#pragma unroll
    for (int i = 0; i < 2 * K; ++i) ss += dev[i];
  } else {
    ss = ((dev[0] + dev[1]) + (dev[2] + dev[3])) + ((dev[4] + dev[5]) + (dev[6] + dev[7]));
  }
  const double rms = sqrt(ss / K);
  if (rms == 0.0) return false;
  nf = kSqrt2 / rms;
  return true;
}

// Affine model through 3 correspondences: L = [v1 v2][u1 u2]^-1 (u_k = s_k - s_0,
// v_k = d_k - d_0), t = c_d - L c_s.  The reference form, with skimage's normalisation
// scales and its degeneracy test evaluated as written (affine_fit3_fast's fallback).
__device__ __forceinline__ HModel affine_fit3(const Pts& P, const int (&sel)[3]) {
  HModel m;
  m.ok = false;
#pragma unroll
  for (int k = 0; k < 9; ++k) m.h[k] = 0.0;
  double csx, csy, nfs, cdx, cdy, nfd;
  if (!center_normalize<3>(P.sx, P.sy, sel, csx, csy, nfs)) return m;
  if (!center_normalize<3>(P.dx, P.dy, sel, cdx, cdy, nfd)) return m;
  const double u1x = P.sx[sel[1]] - P.sx[sel[0]], u1y = P.sy[sel[1]] - P.sy[sel[0]];
  const double u2x = P.sx[sel[2]] - P.sx[sel[0]], u2y = P.sy[sel[2]] - P.sy[sel[0]];
  const double v1x = P.dx[sel[1]] - P.dx[sel[0]], v1y = P.dy[sel[1]] - P.dy[sel[0]];
  const double v2x = P.dx[sel[2]] - P.dx[sel[0]], v2y = P.dy[sel[2]] - P.dy[sel[0]];
  const double det = u1x * u2y - u2x * u1y;
  if (det == 0.0) return m;
  const double l00 = (v1x * u2y - v2x * u1y) / det;
  const double l01 = (v2x * u1x - v1x * u2x) / det;
  const double l10 = (v1y * u2y - v2y * u1y) / det;
  const double l11 = (v2y * u1x - v1y * u2x) / det;
  const double g = nfd / nfs;
  const double hn2 = g * g * (((l00 * l00 + l01 * l01) + l10 * l10) + l11 * l11);
  if (1.0 / sqrt(1.0 + hn2) <= 1e-8) return m;
  m.h[0] = l00;
  m.h[1] = l01;
  m.h[2] = cdx - (l00 * csx + l01 * csy);
  m.h[3] = l10;
  m.h[4] = l11;
  m.h[5] = cdy - (l10 * csx + l11 * csy);
  m.h[8] = 1.0;
  m.ok = true;
  return m;
}

// RN(a / 3) for 2^-600 <= |a| <= 2^600: q = RN(a y) with y = RN(1/3) is within an ulp of
// a / 3, the residual a - 3 q is exact (fma), and RN(q + r y) is then the correctly rounded
// quotient (Markstein); checked bit for bit against a / 3.0 on 4e8 doubles on the host.
// At a == 0, a * y keeps the sign of the zero like the division.
__device__ __forceinline__ double div3(double a) {
  constexpr double y = 1.0 / 3.0;
  const double q = a * y;
  return a == 0.0 ? q : fma(fma(-q, 3.0, a), y, q);
}
__device__ __forceinline__ bool div_operand_ok(double a) {
  const double m = fabs(a);
  return m == 0.0 || (m >= 0x1p-600 && m <= 0x1p600);
}

// a / b for a reciprocal y = recip_newton(b) of 2^-60 <= |b| <= 2^60 and |a| in
// div_operand_ok's range: the compiler's IEEE division sequence (v_div_scale leaves such
// operands unscaled, v_div_fmas is then an fma, v_div_fixup changes nothing but the zero
// numerator, whose signed zero a * y gives), so the same bits; one reciprocal serves every
// numerator over the same b.
__device__ __forceinline__ double recip_newton(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double div_by(double a, double b, double y) {
  const double q = a * y;
  return a == 0.0 ? q : fma(fma(-b, q, a), y, q);
}

// The same model with the per-trial divisions and square roots of the reference form
// removed (round 3; the fit was ~40 % of the f64 work of a c3 trial): the four means by
// div3, the four quotients by det through one reciprocal, skimage's rms == 0 tests as
// sum-of-squares <= 2^-1074 (sqrt(ss / 3) == 0 exactly there), and its
// np.isclose(V[-1,-1], 0) test (1/sqrt(1 + g^2 |L|^2) <= 1e-8, g = nf_d / nf_s) decided
// from g^2 ~ ss_s / ss_d: far below 1e16 it cannot hold.  Any operand outside the ranges
// above, or |L|^2 g^2 >= 1e14, sets need_exact: the caller takes the reference form
// (kept out of the scoring loop, whose registers it would otherwise share).  Bit-identical
// models.
__device__ __forceinline__ HModel affine_fit3_fast(const Pts& P, const int (&sel)[3], bool& need_exact) {
  need_exact = false;
  const double x0 = P.sx[sel[0]], x1 = P.sx[sel[1]], x2 = P.sx[sel[2]];
  const double y0 = P.sy[sel[0]], y1 = P.sy[sel[1]], y2 = P.sy[sel[2]];
  const double p0 = P.dx[sel[0]], p1 = P.dx[sel[1]], p2 = P.dx[sel[2]];
  const double q0 = P.dy[sel[0]], q1 = P.dy[sel[1]], q2 = P.dy[sel[2]];
  // center_normalize's sums: ((0 + v0) + v1) + v2
  double sx = 0.0, sy = 0.0, sp = 0.0, sq = 0.0;
  sx += x0; sx += x1; sx += x2;
  sy += y0; sy += y1; sy += y2;
  sp += p0; sp += p1; sp += p2;
  sq += q0; sq += q1; sq += q2;
  HModel m;
  m.ok = false;
#pragma unroll
  for (int k = 0; k < 9; ++k) m.h[k] = 0.0;
  if (!(div_operand_ok(sx) && div_operand_ok(sy) && div_operand_ok(sp) && div_operand_ok(sq))) {
    need_exact = true;
    return m;
  }
  const double csx = div3(sx), csy = div3(sy), cdx = div3(sp), cdy = div3(sq);
  auto ss6 = [](double a0, double a1, double a2, double b0, double b1, double b2, double ca, double cb) {
    const double e0 = a0 - ca, f0 = b0 - cb, e1 = a1 - ca, f1 = b1 - cb, e2 = a2 - ca, f2 = b2 - cb;
    double ss = 0.0;  // dev order (x0, y0, x1, y1, x2, y2), sequential (2K < 8)
    ss += e0 * e0; ss += f0 * f0; ss += e1 * e1; ss += f1 * f1; ss += e2 * e2; ss += f2 * f2;
    return ss;
  };
  const double ss_s = ss6(x0, x1, x2, y0, y1, y2, csx, csy);
  if (ss_s <= 0x1p-1074) return m;  // rms == 0: ZeroDivisionError in skimage, no model
  const double ss_d = ss6(p0, p1, p2, q0, q1, q2, cdx, cdy);
  if (ss_d <= 0x1p-1074) return m;
  const double u1x = x1 - x0, u1y = y1 - y0, u2x = x2 - x0, u2y = y2 - y0;
  const double v1x = p1 - p0, v1y = q1 - q0, v2x = p2 - p0, v2y = q2 - q0;
  const double det = u1x * u2y - u2x * u1y;
  if (det == 0.0) return m;
  const double n00 = v1x * u2y - v2x * u1y, n01 = v2x * u1x - v1x * u2x;
  const double n10 = v1y * u2y - v2y * u1y, n11 = v2y * u1x - v1y * u2x;
  const double adet = fabs(det);
  if (!(adet >= 0x1p-60 && adet <= 0x1p60 && div_operand_ok(n00) && div_operand_ok(n01) && div_operand_ok(n10) &&
        div_operand_ok(n11))) {
    need_exact = true;
    return m;
  }
  const double y = recip_newton(det);
  const double l00 = div_by(n00, det, y), l01 = div_by(n01, det, y);
  const double l10 = div_by(n10, det, y), l11 = div_by(n11, det, y);
  const double L2 = ((l00 * l00 + l01 * l01) + l10 * l10) + l11 * l11;
  if (!(L2 * (ss_s * __builtin_amdgcn_rcp(ss_d)) < 1e14)) {
    need_exact = true;
    return m;
  }
  m.h[0] = l00;
  m.h[1] = l01;
  m.h[2] = cdx - (l00 * csx + l01 * csy);
  m.h[3] = l10;
  m.h[4] = l11;
  m.h[5] = cdy - (l10 * csx + l11 * csy);
  m.h[8] = 1.0;
  m.ok = true;
  return m;
}

// H = inv(N_dst) Hn N_src with N = [[nf, 0, -nf c_x], [0, nf, -nf c_y], [0, 0, 1]] and
// Hn = [[h0 h1 h2] [h3 h4 h5] [h6 h7 1]] (skimage _geometric.py:699).
__device__ __forceinline__ void denormalize(const double (&h)[8], double csx, double csy, double nfs, double cdx,
                                            double cdy, double nfd, double (&H)[9]) {
  double T[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const double a = h[3 * r], b = h[3 * r + 1], c = (r == 2) ? 1.0 : h[(3 * r + 2) % 8];
    T[3 * r] = a * nfs;
    T[3 * r + 1] = b * nfs;
    T[3 * r + 2] = c - (a * nfs * csx + b * nfs * csy);
  }
  const double id = 1.0 / nfd;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    H[k] = T[k] * id + cdx * T[6 + k];
    H[3 + k] = T[3 + k] * id + cdy * T[6 + k];
    H[6 + k] = T[6 + k];
  }
}

// Projective model through 4 correspondences, in skimage's normalised coordinates:
// rows = the four x-equations then the four y-equations of its A matrix,
//   xs h0 + ys h1 + h2 - xd xs h6 - xd ys h7 = xd,  xs h3 + ys h4 + h5 - yd xs h6 - yd ys h7 = yd.
__device__ __forceinline__ HModel projective_fit4(const Pts& P, const int (&sel)[4]) {
  HModel m;
  m.ok = false;
#pragma unroll
  for (int k = 0; k < 9; ++k) m.h[k] = 0.0;
  double csx, csy, nfs, cdx, cdy, nfd;
  if (!center_normalize<4>(P.sx, P.sy, sel, csx, csy, nfs)) return m;
  if (!center_normalize<4>(P.dx, P.dy, sel, cdx, cdy, nfd)) return m;
  double M[8][9];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double xs = (P.sx[sel[i]] - csx) * nfs, ys = (P.sy[sel[i]] - csy) * nfs;
    const double xd = (P.dx[sel[i]] - cdx) * nfd, yd = (P.dy[sel[i]] - cdy) * nfd;
    M[i][0] = xs;
    M[i][1] = ys;
    M[i][2] = 1.0;
    M[i][3] = 0.0;
    M[i][4] = 0.0;
    M[i][5] = 0.0;
    M[i][6] = -(xd * xs);
    M[i][7] = -(xd * ys);
    M[i][8] = xd;
    M[4 + i][0] = 0.0;
    M[4 + i][1] = 0.0;
    M[4 + i][2] = 0.0;
    M[4 + i][3] = xs;
    M[4 + i][4] = ys;
    M[4 + i][5] = 1.0;
    M[4 + i][6] = -(yd * xs);
    M[4 + i][7] = -(yd * ys);
    M[4 + i][8] = yd;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    int piv = c;
    double best = fabs(M[c][c]);
#pragma unroll
    for (int r = c + 1; r < 8; ++r) {
      const double a = fabs(M[r][c]);
      if (a > best) {
        best = a;
        piv = r;
      }
    }
    if (best == 0.0) return m;
#pragma unroll
    for (int r = c + 1; r < 8; ++r) {
      if (r == piv) {
#pragma unroll
        for (int k = c; k < 9; ++k) {
          const double t = M[c][k];
          M[c][k] = M[r][k];
          M[r][k] = t;
        }
      }
    }
#pragma unroll
    for (int r = c + 1; r < 8; ++r) {
      const double f = M[r][c] / M[c][c];
#pragma unroll
      for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
    }
  }
  double h[8];
#pragma unroll
  for (int c = 7; c >= 0; --c) {
    double v = M[c][8];
#pragma unroll
    for (int k = c + 1; k < 8; ++k) v -= M[c][k] * h[k];
    h[c] = v / M[c][c];
  }
  double hn2 = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) hn2 += h[k] * h[k];
  if (1.0 / sqrt(1.0 + hn2) <= 1e-8) return m;
  denormalize(h, csx, csy, nfs, cdx, cdy, nfd, m.h);
  m.ok = true;
  return m;
}

template <int MODEL>
__device__ __forceinline__ double resid2(const double (&h)[9], const Pts& P, int k, double thresh, int& cnt) {
  const double x = P.sx[k], y = P.sy[k];
  double X = fma(y, h[1], x * h[0]) + h[2];
  double Y = fma(y, h[4], x * h[3]) + h[5];
  if (MODEL == KCMC_MODEL_PROJECTIVE) {
    double w = fma(y, h[7], x * h[6]) + h[8];
    if (w == 0.0) w = DBL_EPSILON;
    X = X / w;
    Y = Y / w;
  }
  const double ex = X - P.dx[k], ey = Y - P.dy[k];
  const double r = sqrt_resid(ex * ex + ey * ey);
  cnt += (r < thresh) ? 1 : 0;
  return r * r;
}

template <int MODEL>
__device__ __forceinline__ double pw_leaf(const double (&h)[9], const Pts& P, int start, int n, double thresh,
                                          int& cnt) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += resid2<MODEL>(h, P, start + i, thresh, cnt);
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = resid2<MODEL>(h, P, start + j, thresh, cnt);
  int i = 8;
  const int nfull = n - (n % 8);
  for (; i < nfull; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += resid2<MODEL>(h, P, start + i + j, thresh, cnt);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += resid2<MODEL>(h, P, start + i, thresh, cnt);
  return res;
}

// Phase A of the scoring (the rigid kernel's, ransac.hip): the exact inlier count through
// q < tq (q computed as resid2 computes it) and the estimate Sd = sum q_k, summed in
// sequence in fp64 (round 6; was an fp32 sum of (float)q_k): within sd_eps(N) of numpy's S,
// so phase B re-scores only trials tied to ~1e-14 instead of ~1e-5 (one fp64 add per point
// in place of a conversion and an fp32 add).
template <int MODEL>
__device__ __forceinline__ double score_fast(const double (&h)[9], const Pts& P, int N, double tq, int& cnt) {
  double S = 0.0;
  for (int k = 0; k < N; ++k) {
    const double x = P.sx[k], y = P.sy[k];
    double X = fma(y, h[1], x * h[0]) + h[2];
    double Y = fma(y, h[4], x * h[3]) + h[5];
    if (MODEL == KCMC_MODEL_PROJECTIVE) {
      double w = fma(y, h[7], x * h[6]) + h[8];
      if (w == 0.0) w = DBL_EPSILON;
      X = X / w;
      Y = Y / w;
    }
    const double ex = X - P.dx[k], ey = Y - P.dy[k];
    const double q = ex * ex + ey * ey;
    cnt += (q < tq) ? 1 : 0;
    S += q;
  }
  return S;
}

// The same over the frame's points packed as (x, y, dx, dy) in LDS (frames with N <= 128):
// two ds_read_b128 with immediate offsets per point and two points per iteration, so the
// reads of a pair are in flight together (the SoA loop issued four address moves and four
// 8-byte reads per point and waited on each point's reads).  Same operations, same order.
struct __attribute__((aligned(16))) PackedPt {
  double2 s, d;  // (x, y), (dx, dy)
};

template <int MODEL>
__device__ __forceinline__ double score_fast_packed(const double (&h)[9], const PackedPt* __restrict__ pk, int N,
                                                    double tq, int& cnt) {
  double S = 0.0;
  auto one = [&](const PackedPt p) {
    double X = fma(p.s.y, h[1], p.s.x * h[0]) + h[2];
    double Y = fma(p.s.y, h[4], p.s.x * h[3]) + h[5];
    if (MODEL == KCMC_MODEL_PROJECTIVE) {
      double w = fma(p.s.y, h[7], p.s.x * h[6]) + h[8];
      if (w == 0.0) w = DBL_EPSILON;
      X = X / w;
      Y = Y / w;
    }
    const double ex = X - p.d.x, ey = Y - p.d.y;
    const double q = ex * ex + ey * ey;
    cnt += (q < tq) ? 1 : 0;
    S += q;
  };
  int k = 0;
  for (; k + 2 <= N; k += 2) {
    const PackedPt a = pk[k], b = pk[k + 1];
    one(a);
    one(b);
  }
  if (k < N) one(pk[k]);
  return S;
}

// Phase A's fit: affine through affine_fit3_fast (need_exact: the trial must be fitted
// again by fit_trial), projective as fit_trial.
template <int MODEL>
__device__ __forceinline__ HModel fit_trial_fast(const Pts& P, uint64_t pr, bool& need_exact) {
  if constexpr (MODEL == KCMC_MODEL_AFFINE) {
    const int sel[3] = {(int)(pr & 0xffffu), (int)((pr >> 16) & 0xffffu), (int)((pr >> 32) & 0xffffu)};
    return affine_fit3_fast(P, sel, need_exact);
  } else {
    need_exact = false;
    const int sel[4] = {(int)(pr & 0xffffu), (int)((pr >> 16) & 0xffffu), (int)((pr >> 32) & 0xffffu),
                        (int)((pr >> 48) & 0xffffu)};
    return projective_fit4(P, sel);
  }
}

template <int MODEL>
__device__ __forceinline__ HModel fit_trial(const Pts& P, uint64_t pr) {
  if constexpr (MODEL == KCMC_MODEL_AFFINE) {
    const int sel[3] = {(int)(pr & 0xffffu), (int)((pr >> 16) & 0xffffu), (int)((pr >> 32) & 0xffffu)};
    return affine_fit3(P, sel);
  } else {
    const int sel[4] = {(int)(pr & 0xffffu), (int)((pr >> 16) & 0xffffu), (int)((pr >> 32) & 0xffffu),
                        (int)((pr >> 48) & 0xffffu)};
    return projective_fit4(P, sel);
  }
}

__device__ __forceinline__ void gather_point(const double* __restrict__ src, const double* __restrict__ dst,
                                             const int32_t* __restrict__ pt_idx, int src_stride, int f, int p,
                                             double& x, double& y, double& u, double& v) {
  size_t si, di;
  if (pt_idx) {
    const int q = pt_idx[p];
    si = (size_t)f * src_stride + q;
    di = (size_t)q;
  } else {
    si = di = (size_t)p;
  }
  x = src[2 * si];
  y = src[2 * si + 1];
  u = dst[2 * di];
  v = dst[2 * di + 1];
}

// The scoring kernel ends each frame with its refit for the homography (kFusedRefit); the
// affine model runs ransac_model_refit_kernel after the scoring.
template <int MODEL>
constexpr bool kFusedRefit = MODEL == KCMC_MODEL_PROJECTIVE;

// The final total-least-squares fit of one frame by one wave (defined with the refit below).
template <int MODEL, class PointFn, class InlierFn>
__device__ __forceinline__ void refit_frame(int N, int lane, PointFn point, InlierFn inlier, const double (&hyp)[9],
                                            double rate, double* o);

// ---------------------------------------------------------------------- scoring
// LARGE = false: frames with N <= 128 (one pairwise leaf) and the NaN frames;
// LARGE = true: 128 < N <= kMaxN through the split plan.
template <int MODEL, bool LARGE>
__device__ __forceinline__ void ransac_model_score_frame(
    int f, const double* __restrict__ src, const double* __restrict__ dst, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_off, int src_stride, const uint64_t* __restrict__ hyp,
    const int32_t* __restrict__ hyp_off, int hyp_off_len, int T, double thresh, double tq, int n_skip, double rate,
    double* out_params, uint8_t* __restrict__ out_inl, int32_t* __restrict__ out_nin, int32_t* __restrict__ out_best) {
  constexpr int K = MODEL == KCMC_MODEL_AFFINE ? 3 : 4;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int s_cnt[kThreads / 64];
  __shared__ double s_min[kThreads / 64];
  __shared__ int s_best[kThreads / 64 * 2];
  __shared__ double s_bestS[kThreads / 64];
  __shared__ int s_any_zero;
  __shared__ int s_final_t;
  __shared__ int s_final_c;
  __shared__ Plan s_plan;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int p0 = pt_off[f];
  const int N = pt_off[f + 1] - p0;

  const bool skip_frame = N < n_skip || N <= K || N > kMaxN;
  const int hoff = (!skip_frame && N < hyp_off_len) ? hyp_off[N] : -1;
  const bool nan_frame = skip_frame || hoff < 0;
  if (LARGE != (!nan_frame && N > 128)) return;  // the other launch owns this frame
  if (nan_frame) {
    if (tid < 9) out_params[9 * (size_t)f + tid] = NAN;
    for (int k = tid; k < N; k += kThreads) out_inl[p0 + k] = 0;
    if (tid == 0) {
      out_nin[f] = skip_frame ? 0 : -1;  // -1: no hypothesis table was prepared for N
      out_best[f] = -1;
    }
    return;
  }

  // LDS: sx, sy, dx, dy [N] f64 | trial S [T] f64 | [LARGE: stack [kMaxStack][256] f64]
  //      | per-wave leaf values [4][128] f64 | trial count [T] i32 | the winner's inlier mask [N] u8
  double* sx = smem;
  double* sy = sx + N;
  double* dxs = sy + N;
  double* dys = dxs + N;
  // !LARGE: the points again as (x, y, dx, dy) for phase A (16-byte aligned: smem is)
  PackedPt* pk = reinterpret_cast<PackedPt*>(smem + ((4 * N + 1) & ~1));
  double* tS = LARGE ? dys + N : reinterpret_cast<double*>(pk + N);
  double* stk = tS + T;
  double* wvals = stk + (LARGE ? kMaxStack * kThreads : 0);
  int* tC = reinterpret_cast<int*>(wvals + kThreads / 64 * 128);
  uint8_t* sinl = reinterpret_cast<uint8_t*>(tC + T);
  if (LARGE && tid == 0) {
    s_plan.n = 0;
    plan_gen<kPwDepth>(s_plan, 0, N);
  }
  for (int k = tid; k < N; k += kThreads) {
    gather_point(src, dst, pt_idx, src_stride, f, p0 + k, sx[k], sy[k], dxs[k], dys[k]);
    if (!LARGE) pk[k] = PackedPt{make_double2(sx[k], sy[k]), make_double2(dxs[k], dys[k])};
  }
  if (tid == 0) s_any_zero = 0;
  __syncthreads();

  const Pts P{sx, sy, dxs, dys};
  const uint64_t* H = hyp + hoff;

  // ---- two-phase scoring, as the rigid kernel (ransac.hip): phase A = exact counts and
  // fp32 S estimates for every trial; phase B = numpy's pairwise S, one wave per trial,
  // for the trials at the best count whose S can tie the smallest; frames the estimates
  // cannot decide score every trial exactly.
  const bool fast = tq == tq;
  int mcount = -1, flag = fast ? 0 : 1;
  if (fast) {
    bool deferred = false;
    for (int t = tid; t < T; t += kThreads) {
      bool need_exact;
      const HModel m = fit_trial_fast<MODEL>(P, H[t], need_exact);
      int cnt = -1;
      double Sd = NAN;
      if (m.ok) {
        cnt = 0;
        Sd = LARGE ? score_fast<MODEL>(m.h, P, N, tq, cnt) : score_fast_packed<MODEL>(m.h, pk, N, tq, cnt);
        if (!sd_certain(Sd)) flag = 1;
      }
      deferred |= need_exact;
      tC[t] = need_exact ? INT_MIN : cnt;
      tS[t] = Sd;
      mcount = max(mcount, cnt);
    }
    // trials whose fast fit fell outside its ranges (in practice none): the reference fit
    if (deferred) {
      for (int t = tid; t < T; t += kThreads) {
        if (tC[t] != INT_MIN) continue;
        const HModel m = fit_trial<MODEL>(P, H[t]);
        int cnt = -1;
        double Sd = NAN;
        if (m.ok) {
          cnt = 0;
          Sd = LARGE ? score_fast<MODEL>(m.h, P, N, tq, cnt) : score_fast_packed<MODEL>(m.h, pk, N, tq, cnt);
          if (!sd_certain(Sd)) flag = 1;
        }
        tC[t] = cnt;
        tS[t] = Sd;
        mcount = max(mcount, cnt);
      }
    }
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
      const HModel m = fit_trial<MODEL>(P, H[t]);
      int cnt = 0;
      double S = NAN;
      if (m.ok) {
        if (!LARGE) {
          S = pw_leaf<MODEL>(m.h, P, 0, N, thresh, cnt);
        } else {
          int sp = 0;
          for (int l = 0; l < s_plan.n; ++l) {
            stk[sp++ * kThreads + tid] = pw_leaf<MODEL>(m.h, P, s_plan.start[l], s_plan.len[l], thresh, cnt);
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
      // skipped trials (estimate() False) and NaN scores never win; with 0 inliers a
      // trial wins only with S < inf (skimage's strict comparisons against (0, inf))
      const bool valid = m.ok && !isnan(S) && (cnt > 0 || S < INFINITY);
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
    const double eps = sd_eps(N);
    double lm = INFINITY;
    for (int t = tid; t < T; t += kThreads)
      if (tC[t] == mcount) lm = fmin(lm, tS[t] * (1.0 + eps));
    for (int o = 32; o > 0; o >>= 1) lm = fmin(lm, __shfl_xor(lm, o));
    if (lane == 0) s_min[wave] = lm;
    __syncthreads();
    const double minhi = fmin(fmin(s_min[0], s_min[1]), fmin(s_min[2], s_min[3]));
    double* vals = wvals + wave * 128;
    double* wstk = stk + wave * kMaxStack;  // LARGE: the wave's combine stack
    for (int t0 = wave * 64; t0 < T; t0 += kThreads) {
      const int t = t0 + lane;
      uint64_t cand = __ballot(t < T && tC[t] == mcount && tS[t] * (1.0 - eps) <= minhi);
      while (cand) {
        const int tc = t0 + __builtin_ctzll(cand);
        cand &= cand - 1;
        const HModel m = fit_trial<MODEL>(P, H[tc]);  // ok: it has a count
        const double S = wave_pairwise<LARGE>(
            [&](int k) {
              int c = 0;
              return resid2<MODEL>(m.h, P, k, thresh, c);
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
      // skimage stops as soon as the running best has S <= 0 (fit.py:862-869)
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
      ft = t0 < 0 ? INT_MAX : t0;
      fc = c0;
    }
    s_final_t = (ft == INT_MAX) ? -1 : ft;
    s_final_c = (ft == INT_MAX) ? 0 : fc;
  }
  __syncthreads();
  const int best_t = s_final_t;
  const int best_c = s_final_c;

  HModel bm;
  bm.ok = false;
  if (best_t >= 0) bm = fit_trial<MODEL>(P, H[best_t]);
  const bool has_model = bm.ok && best_c > 0;
  for (int k = tid; k < N; k += kThreads) {
    int c = 0;
    if (has_model) resid2<MODEL>(bm.h, P, k, thresh, c);
    out_inl[p0 + k] = (uint8_t)c;
    if constexpr (kFusedRefit<MODEL>) sinl[k] = (uint8_t)c;
  }
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 9; ++k)  // skimage: model None (fit.py:876-879); else the separate refit's input
      if (!has_model || !kFusedRefit<MODEL>) out_params[9 * (size_t)f + k] = has_model ? bm.h[k] : NAN;
    out_nin[f] = has_model ? best_c : 0;
    out_best[f] = best_t;
  }
  // the final fit on the inliers (fit.py:871-875), fused for the homography: one wave, the
  // points and the mask from LDS (c5: the separate refit launch ran after every frame's
  // scoring, beside the next slab's match; 92.5-94.1 k -> 97.6 k frames/s).  The affine
  // model keeps the separate launch: fused, its 7 x 7 system takes the kernel from 124 to
  // 157 VGPRs (3 waves per SIMD) or, held to 128, 108 B of spills (c3 even or slower)
  if constexpr (kFusedRefit<MODEL>) {
    if (has_model) {  // workgroup-uniform
    __syncthreads();  // the mask in LDS
    if (wave == 0)
      refit_frame<MODEL>(
          N, lane,
          [&](int k, double& x, double& y, double& u, double& v) {
            x = sx[k];
            y = sy[k];
            u = dxs[k];
            v = dys[k];
          },
          [&](int k) { return sinl[k] != 0; }, bm.h, rate, out_params + 9 * (size_t)f);
    }
  }
}

// ------------------------------------------------------------------------ refit
// skimage takes the TLS solution from np.linalg.svd of the 2N x n system A (n = 7 affine,
// 9 projective; _geometric.py:596-703).  The refit computes that right singular vector from
// A itself, never from A^T A (whose smallest eigenvector carries the square of A's
// condition number: the round-5 inverse iteration on A^T A missed skimage by up to 1e-3 on
// a near-degenerate homography, and stalled on nearly equal singular values):
//   1. Householder QR of A in the wave: each lane holds the two rows of up to P point pairs
//      (chunks of 64 P pairs) and, in lanes 0..n-1, one row of the running triangle R;
//      column j's reflection takes n - j wave sums;
//   2. inverse iteration on R^T R (two triangular solves with R per step; pivots floored at
//      |R|_F 2^-52) while it converges (successive iterates within 1e-15, at most 40 steps);
//   3. otherwise (nearly equal smallest singular values) a one-sided Jacobi SVD of R, one row
//      of R and of V per lane: V's column of the smallest R V column norm.
// tools/debug/refit_spread.py restates all three in numpy: within 1e-11 of skimage on every
// fuzz case of the GPU sweeps, where LAPACK's own drivers spread by ~1e-12.
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Sum over the 16 lanes of a DPP row: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror.  Each step adds a partner's value to one's own, so every lane of the row ends
// with the bitwise same sum (a + b == b + a).
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return v;
}

// Sum over the wave, the same value in every lane: the four row sums read from lanes 0, 16,
// 32 and 48.
__device__ __forceinline__ double wave_sum_u(double v) {
  v = row16_sum(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// One chunk of the Householder QR: the rows are the S data rows m[0..S-1] of every lane and,
// in lanes 0..n-1, the triangle's row rr (row index = lane; rows < j are final at step j).
// Column j is reflected onto lane j's rr[j] (LAPACK's sign: beta = -sign(x_j) |x|).
template <int n, int S>
__device__ __forceinline__ void householder_chunk(double (&m)[S][n], double (&rr)[n], int lane) {
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const bool ract = lane >= j && lane < n;
    const double xr = ract ? rr[j] : 0.0;
    double part = xr * xr;
#pragma unroll
    for (int s = 0; s < S; ++s) part += m[s][j] * m[s][j];
    const double alpha = wave_sum_u(part);
    if (alpha == 0.0) continue;  // the column is zero below the diagonal: R[j][j] = 0 (uniform)
    const double xj = readlane_d(rr[j], j);
    const double nx = sqrt(alpha);
    const double beta = xj >= 0.0 ? -nx : nx;
    const double f2 = 1.0 / (alpha - beta * xj);  // 2 / v^T v, v = x - beta e_j
    const double vr = lane == j ? xj - beta : xr;
    double dot[n];
#pragma unroll
    for (int c = j + 1; c < n; ++c) {
      double d = ract ? vr * rr[c] : 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s) d += m[s][j] * m[s][c];
      dot[c] = d;
    }
#pragma unroll
    for (int c = j + 1; c < n; ++c) dot[c] = wave_sum_u(dot[c]) * f2;
#pragma unroll
    for (int c = j + 1; c < n; ++c) {
      if (ract) rr[c] -= vr * dot[c];
#pragma unroll
      for (int s = 0; s < S; ++s) m[s][c] -= m[s][j] * dot[c];
    }
    if (lane == j) rr[j] = beta;
    else if (ract) rr[j] = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) m[s][j] = 0.0;
  }
}

// One-sided (Hestenes) Jacobi on the n x n R held one row per lane (lane & 15 = row; rows
// >= n zero; the four DPP rows of the wave identical, so every branch is uniform).  Returns
// in v, in every lane, the column of V whose column of R V has the smallest norm.
template <int n>
__device__ __forceinline__ void jacobi_smallest(double (&rr)[n], double (&vr)[n], double (&v)[n]) {
  for (int sweep = 0; sweep < 30; ++sweep) {
    double nrm[n];
#pragma unroll
    for (int j = 0; j < n; ++j) nrm[j] = row16_sum(rr[j] * rr[j]);
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < n - 1; ++p)
#pragma unroll
      for (int q = p + 1; q < n; ++q) {
        const double g = row16_sum(rr[p] * rr[q]);
        const double a = nrm[p], b = nrm[q];
        if (fabs(g) > 7.105427357601002e-15 * sqrt(fmax(a * b, 0.0))) {  // 32 eps: above a dot's rounding
          const double zeta = (b - a) / (2.0 * g);
          const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
          const double rp = rr[p], rq = rr[q], vp = vr[p], vq = vr[q];
          rr[p] = c * rp - s * rq;
          rr[q] = s * rp + c * rq;
          vr[p] = c * vp - s * vq;
          vr[q] = s * vp + c * vq;
          nrm[p] = a - t * g;
          nrm[q] = b + t * g;
          rotated = true;
        }
      }
    if (!rotated) break;
  }
  int js = 0;
  double best = INFINITY;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const double q = row16_sum(rr[j] * rr[j]);
    if (q < best) {
      best = q;
      js = j;
    }
  }
  double mine = 0.0;
#pragma unroll
  for (int j = 0; j < n; ++j)
    if (j == js) mine = vr[j];
#pragma unroll
  for (int i = 0; i < n; ++i) v[i] = readlane_d(mine, i);
}

// Inverse iteration on R^T R (every lane holds R whole).  Returns false if it has not
// converged in 40 steps (the two smallest singular values nearly equal).
template <int n>
__device__ __forceinline__ bool inverse_iteration(const double (&R)[n][n], double (&x)[n]) {
  double fro = 0.0;
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = i; j < n; ++j) fro += R[i][j] * R[i][j];
  const double floor_v = sqrt(fro) * 2.220446049250313e-16 + DBL_MIN;
  double dinv[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double d = R[i][i];
    if (!(fabs(d) > floor_v)) d = floor_v;
    dinv[i] = 1.0 / d;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) x[i] = 1.0;
  for (int it = 0; it < 40; ++it) {
    double y[n], z[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {  // R^T y = x
      double a = x[i];
#pragma unroll
      for (int k = 0; k < i; ++k) a -= R[k][i] * y[k];
      y[i] = a * dinv[i];
    }
#pragma unroll
    for (int i = n - 1; i >= 0; --i) {  // R z = y
      double a = y[i];
#pragma unroll
      for (int k = i + 1; k < n; ++k) a -= R[i][k] * z[k];
      z[i] = a * dinv[i];
    }
    double nn = 0.0, dt = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      nn += z[i] * z[i];
      dt += z[i] * x[i];
    }
    const double sc = (dt < 0.0 ? -1.0 : 1.0) / sqrt(nn);
    double diff = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const double v = z[i] * sc;
      diff = fmax(diff, fabs(v - x[i]));
      x[i] = v;
    }
    if (it > 0 && diff < 1e-15) return true;
  }
  return false;
}

// The triangle of A's rows (point pairs k = base + lane + 64 i, i < P, inliers only).
template <int MODEL, int P, class PointFn, class InlierFn>
__device__ __forceinline__ void qr_rows(int N, int lane, PointFn point, InlierFn inlier, double csx, double csy,
                                        double nfs, double cdx, double cdy, double nfd,
                                        double (&rr)[MODEL == KCMC_MODEL_AFFINE ? 7 : 9]) {
  constexpr int n = MODEL == KCMC_MODEL_AFFINE ? 7 : 9;
  for (int base = 0; base < N; base += 64 * P) {
    double m[2 * P][n];
#pragma unroll
    for (int i = 0; i < P; ++i) {
#pragma unroll
      for (int c = 0; c < n; ++c) m[2 * i][c] = m[2 * i + 1][c] = 0.0;
      const int k = base + lane + 64 * i;
      if (k < N && inlier(k)) {
        double x, y, u, v;
        point(k, x, y, u, v);
        const double xs = (x - csx) * nfs, ys = (y - csy) * nfs;
        const double e = (u - cdx) * nfd, g = (v - cdy) * nfd;
        // skimage's rows (_geometric.py:665-680): (s, 0, -e xs, -e ys, e), (0, s, -g xs, -g ys, g)
        // with s = (xs, ys, 1); the affine system keeps columns 0-5 and 8
        m[2 * i][0] = m[2 * i + 1][3] = xs;
        m[2 * i][1] = m[2 * i + 1][4] = ys;
        m[2 * i][2] = m[2 * i + 1][5] = 1.0;
        if constexpr (MODEL == KCMC_MODEL_AFFINE) {
          m[2 * i][6] = e;
          m[2 * i + 1][6] = g;
        } else {
          m[2 * i][6] = -e * xs;
          m[2 * i][7] = -e * ys;
          m[2 * i][8] = e;
          m[2 * i + 1][6] = -g * xs;
          m[2 * i + 1][7] = -g * ys;
          m[2 * i + 1][8] = g;
        }
      }
    }
    householder_chunk<n, 2 * P>(m, rr, lane);
  }
}

// Workgroup g scores frames g, g + grid, ... (the product launches one per frame).
// (projective: 2 waves per SIMD, its scoring alone needs 231 VGPRs)
template <int MODEL, bool LARGE>
__global__ __launch_bounds__(kThreads, MODEL == KCMC_MODEL_AFFINE ? 1 : 2) void
ransac_model_score_kernel(
    int n_frames, const double* __restrict__ src, const double* __restrict__ dst, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_off, int src_stride, const uint64_t* __restrict__ hyp,
    const int32_t* __restrict__ hyp_off, int hyp_off_len, int T, double thresh, double tq, int n_skip, double rate,
    double* out_params, uint8_t* __restrict__ out_inl, int32_t* __restrict__ out_nin,
    int32_t* __restrict__ out_best) {
  for (int f = blockIdx.x; f < n_frames; f += gridDim.x) {
    ransac_model_score_frame<MODEL, LARGE>(f, src, dst, pt_idx, pt_off, src_stride, hyp, hyp_off, hyp_off_len, T,
                                           thresh, tq, n_skip, rate, out_params, out_inl, out_nin, out_best);
    __syncthreads();  // the frame's LDS is free for the next one
  }
}

// The affine model's refit after the scoring: one wave per frame, the points through pt_idx
// and the mask from global memory; the hypothesis model is the scoring's out_params entry,
// overwritten here.
template <int MODEL>
__global__ __launch_bounds__(256) void ransac_model_refit_kernel(
    const double* __restrict__ src, const double* __restrict__ dst, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_off, int src_stride, const uint8_t* __restrict__ inl,
    const int32_t* __restrict__ nin, int n_frames, double rate, double* out_params) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (f >= n_frames || nin[f] <= 0) return;  // NaN params already written by the scoring kernel
  const int p0 = pt_off[f], N = pt_off[f + 1] - p0;
  double* o = out_params + 9 * (size_t)f;
  double hyp[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) hyp[k] = o[k];
  refit_frame<MODEL>(
      N, lane,
      [&](int k, double& x, double& y, double& u, double& v) {
        gather_point(src, dst, pt_idx, src_stride, f, p0 + k, x, y, u, v);
      },
      [&](int k) { return inl[p0 + k] != 0; }, hyp, rate, o);
}

// The final fit of one frame by one wave (lane = its lane): point(k, x, y, u, v) gives
// point pair k of the frame's N, inlier(k) its mask entry, hyp the scoring's model (kept
// when the refit is degenerate); the result, scaled by the spatial rate, goes to o[0..8].
template <int MODEL, class PointFn, class InlierFn>
__device__ __forceinline__ void refit_frame(int N, int lane, PointFn point, InlierFn inlier, const double (&hyp)[9],
                                            double rate, double* o) {
  constexpr int n = MODEL == KCMC_MODEL_AFFINE ? 7 : 9;

  // centroids (np.mean(points, axis=0) of the inliers)
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, sc = 0.0;
  for (int k = lane; k < N; k += 64)
    if (inlier(k)) {
      double x, y, u, v;
      point(k, x, y, u, v);
      s0 += x;
      s1 += y;
      s2 += u;
      s3 += v;
      sc += 1.0;
    }
  const double cnt = wave_sum(sc);
  const double csx = wave_sum(s0) / cnt, csy = wave_sum(s1) / cnt;
  const double cdx = wave_sum(s2) / cnt, cdy = wave_sum(s3) / cnt;
  double q0 = 0.0, q1 = 0.0;
  for (int k = lane; k < N; k += 64)
    if (inlier(k)) {
      double x, y, u, v;
      point(k, x, y, u, v);
      q0 += (x - csx) * (x - csx) + (y - csy) * (y - csy);
      q1 += (u - cdx) * (u - cdx) + (v - cdy) * (v - cdy);
    }
  const double rms_s = sqrt(wave_sum(q0) / cnt), rms_d = sqrt(wave_sum(q1) / cnt);
  if (rms_s == 0.0 || rms_d == 0.0) {  // skimage: ZeroDivisionError -> params = NaN
    if (lane < 9) o[lane] = NAN;
    return;
  }
  const double nfs = kSqrt2 / rms_s, nfd = kSqrt2 / rms_d;

  // 1. QR: lane i (< n) ends with row i of R
  double rr[n];
#pragma unroll
  for (int j = 0; j < n; ++j) rr[j] = 0.0;
  if (N <= 64)
    qr_rows<MODEL, 1>(N, lane, point, inlier, csx, csy, nfs, cdx, cdy, nfd, rr);
  else
    qr_rows<MODEL, 2>(N, lane, point, inlier, csx, csy, nfs, cdx, cdy, nfd, rr);
  // 2. R in every lane, inverse iteration on it
  double R[n][n];
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j < n; ++j) R[i][j] = j >= i ? readlane_d(rr[j], i) : 0.0;
  double v[n];
  if (!inverse_iteration<n>(R, v)) {
    // 3. nearly equal smallest singular values: Jacobi SVD of R (row lane & 15 in every DPP row)
    const int my = lane & 15;
    double jr[n], jv[n];
#pragma unroll
    for (int j = 0; j < n; ++j) {
      double r = 0.0;
#pragma unroll
      for (int i = 0; i < n; ++i)
        if (i == my) r = R[i][j];
      jr[j] = r;
      jv[j] = j == my ? 1.0 : 0.0;
    }
    jacobi_smallest<n>(jr, jv, v);
  }
  double Hm[9];
  if (fabs(v[n - 1]) <= 1e-8) {
    // np.isclose(V[-1, -1], 0): estimate() returns False and keeps the hypothesis model
#pragma unroll
    for (int k = 0; k < 9; ++k) Hm[k] = hyp[k];
  } else {
    double h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = 0.0;
#pragma unroll
    for (int k = 0; k < n - 1; ++k) h[k] = -v[k] / v[n - 1];
    denormalize(h, csx, csy, nfs, cdx, cdy, nfd, Hm);
  }
  if (lane == 0) {
    o[0] = Hm[0];
    o[1] = Hm[1];
    o[2] = Hm[2] * rate;
    o[3] = Hm[3];
    o[4] = Hm[4];
    o[5] = Hm[5] * rate;
    o[6] = Hm[6] / rate;
    o[7] = Hm[7] / rate;
    o[8] = Hm[8];
  }
}


}  // namespace
}  // namespace kcmc

using namespace kcmc;

static int ransac_model_impl(kcmc_ctx* ctx, int model, const double* src, const double* dst,
                                 const int32_t* pt_idx, const int32_t* pt_off, int src_frame_stride, int n_frames,
                                 int max_n, int trials, double thresh, double rate, int n_skip, double* out_params,
                                 uint8_t* out_inliers, int32_t* out_n_inliers, int32_t* out_best_trial,
                                 int max_workgroups, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_ransac_model: ctx is NULL");
  if (model != KCMC_MODEL_AFFINE && model != KCMC_MODEL_PROJECTIVE)
    return fail(KCMC_EINVAL, "kcmc_ransac_model: model must be KCMC_MODEL_AFFINE or KCMC_MODEL_PROJECTIVE "
                             "(the Euclidean model is kcmc_ransac_rigid)");
  if (n_frames < 0 || max_n < 0 || trials < 1) return fail(KCMC_EINVAL, "kcmc_ransac_model: bad sizes");
  if (!(rate > 0.0)) return fail(KCMC_EINVAL, "kcmc_ransac_model: spatial_rate must be > 0");
  if (n_frames == 0) return KCMC_OK;
  if (!pt_off || !out_params || !out_n_inliers || !out_best_trial || (max_n > 0 && (!src || !dst || !out_inliers)))
    return fail(KCMC_EINVAL, "kcmc_ransac_model: NULL pointer");
  if (max_n > kMaxN) return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_model: max_n > 4096 points per frame");
  if (pt_idx && src_frame_stride <= 0) return fail(KCMC_EINVAL, "kcmc_ransac_model: src_frame_stride must be > 0");
  const int ms = model == KCMC_MODEL_AFFINE ? 3 : 4;
  const HypTables& tab = ctx->mhyp[ms];
  if (!tab.dev || tab.trials != trials)
    return fail(KCMC_EINVAL, "kcmc_ransac_model: hypothesis tables not prepared for min_samples=" +
                                 std::to_string(ms) + ", trials=" + std::to_string(trials) +
                                 " (call kcmc_ransac_prepare_samples)");
  const int need = max_n < ms + 1 ? ms + 1 : max_n;
  const int n_small = need < 128 ? need : 128;
  const size_t wvals = (size_t)kThreads / 64 * 128 * sizeof(double);
  // + the winner's inlier mask (N bytes) for the fused refit
  const size_t lds_small = (size_t)(n_small + 1) * 4 * sizeof(double) + (size_t)n_small * 4 * sizeof(double) +
                           (size_t)trials * (sizeof(double) + sizeof(int)) + wvals + 16 + (((size_t)n_small + 15) & ~15);
  const size_t lds_large = (size_t)need * 4 * sizeof(double) + (size_t)trials * (sizeof(double) + sizeof(int)) + wvals +
                           (size_t)kMaxStack * kThreads * sizeof(double) + 16 + (((size_t)need + 15) & ~15);
  if ((max_n > 128 ? lds_large : lds_small) > 150 * 1024)
    return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_model: max_n/trials exceed the LDS budget");
  const double tq = inlier_bound(thresh);
  hipStream_t s = (hipStream_t)stream;
  // The scoring kernel writes out_params: the homography's refit is fused into it (one wave
  // per frame, points and mask from LDS); the affine model's hypothesis model goes there
  // first and ransac_model_refit_kernel overwrites it with the refit.  No workspace: a stream-ordered pool allocation cost
  // ~0.2 ms of host time per call.
  const unsigned grid = (unsigned)(max_workgroups > 0 && max_workgroups < n_frames ? max_workgroups : n_frames);
  if (model == KCMC_MODEL_AFFINE) {
    hipLaunchKernelGGL((ransac_model_score_kernel<KCMC_MODEL_AFFINE, false>), dim3(grid), dim3(kThreads),
                       lds_small, s, n_frames, src, dst, pt_idx, pt_off, src_frame_stride, tab.dev, tab.off, tab.off_len,
                       trials, thresh, tq, n_skip, rate, out_params, out_inliers, out_n_inliers, out_best_trial);
    if (max_n > 128)
      hipLaunchKernelGGL((ransac_model_score_kernel<KCMC_MODEL_AFFINE, true>), dim3(grid), dim3(kThreads),
                         lds_large, s, n_frames, src, dst, pt_idx, pt_off, src_frame_stride, tab.dev, tab.off, tab.off_len,
                         trials, thresh, tq, n_skip, rate, out_params, out_inliers, out_n_inliers, out_best_trial);
    hipLaunchKernelGGL((ransac_model_refit_kernel<KCMC_MODEL_AFFINE>), dim3((unsigned)ceil_div(n_frames, 4)), dim3(256),
                       0, s, src, dst, pt_idx, pt_off, src_frame_stride, out_inliers, out_n_inliers, n_frames, rate,
                       out_params);
  } else {
    hipLaunchKernelGGL((ransac_model_score_kernel<KCMC_MODEL_PROJECTIVE, false>), dim3(grid), dim3(kThreads),
                       lds_small, s, n_frames, src, dst, pt_idx, pt_off, src_frame_stride, tab.dev, tab.off, tab.off_len,
                       trials, thresh, tq, n_skip, rate, out_params, out_inliers, out_n_inliers, out_best_trial);
    if (max_n > 128)
      hipLaunchKernelGGL((ransac_model_score_kernel<KCMC_MODEL_PROJECTIVE, true>), dim3(grid), dim3(kThreads),
                         lds_large, s, n_frames, src, dst, pt_idx, pt_off, src_frame_stride, tab.dev, tab.off, tab.off_len,
                         trials, thresh, tq, n_skip, rate, out_params, out_inliers, out_n_inliers, out_best_trial);
  }
  return launch_check("ransac_model kernels");
}

extern "C" int kcmc_ransac_model(kcmc_ctx* ctx, int model, const double* src, const double* dst,
                                 const int32_t* pt_idx, const int32_t* pt_off, int src_frame_stride, int n_frames,
                                 int max_n, int trials, double thresh, double rate, int n_skip, double* out_params,
                                 uint8_t* out_inliers, int32_t* out_n_inliers, int32_t* out_best_trial,
                                 kcmc_stream_t stream) {
  return ransac_model_impl(ctx, model, src, dst, pt_idx, pt_off, src_frame_stride, n_frames, max_n, trials, thresh, rate, n_skip, out_params, out_inliers, out_n_inliers, out_best_trial, 0, stream);
}
