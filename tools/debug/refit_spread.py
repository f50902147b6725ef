"""The projective / affine refit's accuracy on one fuzz case (CPU only, no GPU): the
total-least-squares system skimage solves (_geometric.py:596-703, fit.py:871-875) on the
winner's inliers, solved by

  * numpy.linalg.svd                      (skimage's own call: LAPACK gesdd)
  * scipy.linalg.svd(lapack_driver=gesvd) (another LAPACK driver)
  * numpy.linalg.eigh(A^T A)              (the normal equations, a LAPACK eigensolver)
  * chol_inv_iter(A^T A)                  (the round-5 GPU refit: Cholesky inverse iteration on A^T A)
  * givens_qr_inv_iter(A)                 (Givens QR of A, per-lane triangles merged in a
                                           tree, inverse iteration on R: not adopted)
  * givens_qr_jacobi(A)                   (the same QR, then a one-sided Jacobi SVD of R)
  * householder_hybrid(A)                 (the round-6 GPU refit: Householder QR of A in chunks
                                           of 64 P point pairs, inverse iteration on R for at
                                           most 40 steps, else the Jacobi SVD of R)

and the difference of each model H against skimage's, per entry as the GPU tests measure
it: max |dH| / (|H| + 0.1 max(1, |dst|)) (the ratio of the tests' atol to their rtol), next
to the spread of LAPACK itself on the same problem (gesvd, and gesdd on the rows mixed by a
random orthogonal matrix -- the same TLS problem, rounded differently).

    python tools/debug/refit_spread.py [seed] [frame] [model]       (default: 20410 3 projective)
"""
import os
import sys

import numpy as np
import scipy.linalg

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "oracle"), os.path.join(R, "tests")]
import oracle  # noqa: E402
import test_gpu_fuzz as T  # noqa: E402

COLS = {"affine": [0, 1, 2, 3, 4, 5, 8], "projective": list(range(9))}


def system(src, dst, model):
    Ns, s = oracle._center_and_normalize(np.asarray(src, np.float64))
    Nd, d = oracle._center_and_normalize(np.asarray(dst, np.float64))
    xs, ys, xd, yd = s[:, 0], s[:, 1], d[:, 0], d[:, 1]
    n = len(s)
    A = np.zeros((2 * n, 9))
    A[:n, 0], A[:n, 1], A[:n, 2] = xs, ys, 1
    A[n:, 3], A[n:, 4], A[n:, 5] = xs, ys, 1
    A[:n, 6], A[:n, 7], A[:n, 8] = -xd * xs, -xd * ys, xd
    A[n:, 6], A[n:, 7], A[n:, 8] = -yd * xs, -yd * ys, yd
    if model == "affine":
        A[:, 6], A[:, 7] = 0, 0
    return A[:, COLS[model]], Ns, Nd


def model_from(v, Ns, Nd, model):
    H = np.zeros((3, 3))
    H.flat[COLS[model][:-1]] = -v[:-1] / v[-1]
    H[2, 2] = 1
    return np.linalg.inv(Nd) @ H @ Ns


def inv_iter(L_solve, n):
    x = np.ones(n)
    for it in range(200):
        z = L_solve(x)
        z = z * ((-1.0 if z @ x < 0 else 1.0) / np.sqrt(z @ z))
        diff = np.abs(z - x).max()
        x = z
        if it > 0 and diff < 1e-15:
            break
    return x


def chol_inv_iter(A):
    """Round 5: pivots floored at trace * 2^-52, inverse iteration with L L^T."""
    M = A.T @ A
    n = len(M)
    fl = np.trace(M) * 2.220446049250313e-16 + np.finfo(float).tiny
    L = np.zeros_like(M)
    for j in range(n):
        d = M[j, j] - L[j, :j] @ L[j, :j]
        L[j, j] = np.sqrt(max(d, fl)) if d > fl else np.sqrt(fl)
        for i in range(j + 1, n):
            L[i, j] = (M[i, j] - L[i, :j] @ L[j, :j]) / L[j, j]
    return inv_iter(lambda x: scipy.linalg.solve_triangular(L.T, scipy.linalg.solve_triangular(L, x, lower=True)), n)


def givens_rows(Rm, row):
    """Rotate one row into the upper-triangular Rm (in place)."""
    n = len(row)
    row = row.copy()
    for j in range(n):
        b = row[j]
        if b == 0.0:
            continue
        a = Rm[j, j]
        r = np.sqrt(a * a + b * b)
        c, s = a / r, b / r
        rj = Rm[j, j:].copy()
        Rm[j, j:] = c * rj + s * row[j:]
        row[j:] = -s * rj + c * row[j:]
        Rm[j, j] = r
        row[j] = 0.0


def givens_qr_inv_iter(A, lanes=64):
    """Lane l triangularises the point pairs k = l, l + 64, ... (both rows of a
    pair), then the lanes' triangles merge pairwise (xor 32, 16, ..., 1) -- as the GPU wave
    does -- and inverse iteration runs on R^T R (pivots floored at |R|_F * 2^-52)."""
    n2, n = A.shape
    N = n2 // 2
    Rs = [np.zeros((n, n)) for _ in range(lanes)]
    for k in range(N):
        givens_rows(Rs[k % lanes], A[k])
        givens_rows(Rs[k % lanes], A[N + k])
    off = lanes // 2
    while off:
        new = []
        for l in range(lanes):
            Rm = Rs[l].copy()
            for i in range(n):
                givens_rows(Rm, Rs[l ^ off][i])
            new.append(Rm)
        Rs = new
        off //= 2
    Rm = Rs[0]
    fl = np.sqrt((Rm * Rm).sum()) * 2.220446049250313e-16 + np.finfo(float).tiny
    Rf = Rm.copy()
    for j in range(n):
        if not Rf[j, j] > fl:
            Rf[j, j] = fl
    return inv_iter(lambda x: scipy.linalg.solve_triangular(Rf, scipy.linalg.solve_triangular(Rf.T, x, lower=True)), n)


def one_sided_jacobi(Rm, max_sweeps=30):
    """Hestenes: rotate column pairs of R (and of V = I) until every pair is orthogonal to
    |g| <= 32 eps sqrt(a b); a, b are updated per rotation (a - t g, b + t g) and recomputed
    at each sweep's start.  Returns the column of V whose R-column has the smallest norm."""
    R = Rm.copy()
    n = len(R)
    V = np.eye(n)
    for sweep in range(max_sweeps):
        nrm = (R * R).sum(0)
        rot = 0
        for p in range(n - 1):
            for q in range(p + 1, n):
                g = R[:, p] @ R[:, q]
                a, b = nrm[p], nrm[q]
                if not abs(g) > 7.105427357601002e-15 * np.sqrt(max(a * b, 0.0)):
                    continue
                rot += 1
                zeta = (b - a) / (2.0 * g)
                t = (1.0 if zeta >= 0 else -1.0) / (abs(zeta) + np.sqrt(1.0 + zeta * zeta))
                c = 1.0 / np.sqrt(1.0 + t * t)
                s_ = c * t
                Rp, Rq = R[:, p].copy(), R[:, q].copy()
                R[:, p], R[:, q] = c * Rp - s_ * Rq, s_ * Rp + c * Rq
                Vp, Vq = V[:, p].copy(), V[:, q].copy()
                V[:, p], V[:, q] = c * Vp - s_ * Vq, s_ * Vp + c * Vq
                nrm[p], nrm[q] = a - t * g, b + t * g
        if rot == 0:
            break
    nrm = (R * R).sum(0)
    return V[:, int(np.argmin(nrm))], sweep + 1


def givens_qr(A, lanes=64):
    n2, n = A.shape
    N = n2 // 2
    Rs = [np.zeros((n, n)) for _ in range(lanes)]
    for k in range(N):
        givens_rows(Rs[k % lanes], A[k])
        givens_rows(Rs[k % lanes], A[N + k])
    off = lanes // 2
    while off:
        new = []
        for l in range(lanes):
            Rm = Rs[l].copy()
            for i in range(n):
                givens_rows(Rm, Rs[l ^ off][i])
            new.append(Rm)
        Rs = new
        off //= 2
    return Rs[0]


def givens_qr_jacobi(A):
    return one_sided_jacobi(givens_qr(A))[0]


def householder_r(A, P=None):
    """The GPU's Householder QR: chunks of 64 P point pairs (P = 1 for N <= 64, else 2), the
    running triangle carried as n extra rows; column j reflected onto R[j][j] = -sign(x_j)|x|."""
    n2, n = A.shape
    N = n2 // 2
    P = P or (1 if N <= 64 else 2)
    Rm = np.zeros((n, n))
    for base in range(0, max(N, 1), 64 * P):
        ks = np.arange(base, min(N, base + 64 * P))
        M = np.vstack([Rm, A[ks], A[N + ks]])
        for j in range(n):
            x = M[j:, j].copy()
            alpha = x @ x
            if alpha == 0.0:
                continue
            beta = -np.sqrt(alpha) if x[0] >= 0 else np.sqrt(alpha)
            v = x.copy()
            v[0] -= beta
            f2 = 1.0 / (alpha - beta * x[0])
            M[j:, j + 1:] -= np.outer(v, (v @ M[j:, j + 1:]) * f2)
            M[j, j], M[j + 1:, j] = beta, 0.0
        Rm = M[:n].copy()
    return Rm


def inv_iter_r(Rm, cap=40):
    n = len(Rm)
    fl = np.sqrt((np.triu(Rm) ** 2).sum()) * 2.220446049250313e-16 + np.finfo(float).tiny
    d = np.diag(Rm).copy()
    d[~(np.abs(d) > fl)] = fl
    Rf = np.triu(Rm, 1) + np.diag(d)
    x = np.ones(n)
    for it in range(cap):
        z = scipy.linalg.solve_triangular(Rf, scipy.linalg.solve_triangular(Rf.T, x, lower=True))
        z = z * ((-1.0 if z @ x < 0 else 1.0) / np.sqrt(z @ z))
        diff = np.abs(z - x).max()
        x = z
        if it > 0 and diff < 1e-15:
            return x
    return None


def householder_hybrid(A):
    Rm = householder_r(A)
    v = inv_iter_r(Rm)
    return one_sided_jacobi(Rm)[0] if v is None else v


def rel(H, ref, sc=1.0):
    return float(np.max(np.abs(H - ref) / (np.abs(ref) + 0.1 * max(1.0, sc))))


def lapack_spread(A, Ns, Nd, model, sc, seed=0):
    """How far LAPACK's own answers to this TLS problem spread (test metric)."""
    ref = model_from(np.linalg.svd(A)[2][-1], Ns, Nd, model)
    Q, _ = np.linalg.qr(np.random.default_rng(seed).normal(size=(len(A), len(A))))
    alt = [scipy.linalg.svd(A, lapack_driver="gesvd")[2][-1], np.linalg.svd(Q @ A)[2][-1]]
    return max(rel(model_from(v, Ns, Nd, model), ref, sc) for v in alt)


def case(seed, frame, model):
    rng = np.random.default_rng(4000 + seed + (100 if model == "projective" else 0))
    tpls, qs = T._point_sets(rng, 12, model)
    ms = 3 if model == "affine" else 4
    for f in range(len(qs)):
        if 3 <= len(qs[f]) <= ms:
            tpls[f], qs[f] = tpls[f][:2], qs[f][:2]
    return qs[frame], tpls[frame]


def spread(src, dst, model, verbose=True):
    H_sk, inl, bt, ni = oracle.ransac_model(src, dst, model)
    A, Ns, Nd = system(src[inl], dst[inl], model)
    sv = np.linalg.svd(A, compute_uv=False)
    out = {"n_inliers": int(ni), "rows": A.shape[0], "sv": sv}
    vs = {
        "numpy svd (skimage)": np.linalg.svd(A)[2][-1],
        "scipy gesvd": scipy.linalg.svd(A, lapack_driver="gesvd")[2][-1],
        "numpy eigh(AtA)": np.linalg.eigh(A.T @ A)[1][:, 0],
        "r5 GPU: chol inv-iter on AtA": chol_inv_iter(A),
        "givens QR + inv-iter on R": givens_qr_inv_iter(A),
        "givens QR + jacobi(R)": givens_qr_jacobi(A),
        "r6 GPU: householder + inv-iter / jacobi": householder_hybrid(A),
    }
    ref = model_from(vs["numpy svd (skimage)"], Ns, Nd, model)
    sc = float(np.abs(dst).max()) if len(dst) else 1.0
    for k, v in vs.items():
        out[k] = rel(model_from(v, Ns, Nd, model), ref, sc)
    out["lapack spread"] = lapack_spread(A, Ns, Nd, model, sc)
    if verbose:
        print(f"inliers {ni}  A {A.shape}  singular values {np.array2string(sv, precision=3)}")
        print(f"|H| max {np.abs(ref).max():.3g}   v_last/|v| {abs(vs['numpy svd (skimage)'][-1]):.3g}")
        for k in vs:
            print(f"  {k:38s} diff vs skimage (test metric)  {out[k]:.3g}")
        print(f"  {'LAPACK spread':38s} {out['lapack spread']:.3g}")
    return out


if __name__ == "__main__":
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 20410
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    model = sys.argv[3] if len(sys.argv) > 3 else "projective"
    src, dst = case(seed, frame, model)
    print(f"seed {seed} frame {frame} {model}: N = {len(src)}")
    spread(src, dst, model)
