"""kcmc CPU oracle -- TEST INFRASTRUCTURE ONLY.

Restates, on the CPU, what the reference's per-frame alignment hot path computes
(/root/reference/VideoAligner.py, cited as VA:<line>) so that tests can check the
HIP product path.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product package
(``kcmc_amd``) never does, and fails loudly if its HIP library is missing.

Contents
--------
* ctypes wrappers over ``libkcmc_oracle.so`` (``kcmc_oracle.c``): OpenCV knnMatch
  (NORM_L2, k=2), OpenCV classic warpAffine INTER_LINEAR on uint16, closed-form
  rigid RANSAC with skimage 0.18.3 selection semantics.
* ``hypothesis_table``: the seeded sample stream skimage consumes
  (``np.random.RandomState(42).choice(N, 2, replace=False)`` per trial, skimage
  fit.py:819-826), generated with numpy itself.
* ``ransac_rigid_skimage``: a slow, operation-for-operation numpy restatement of
  skimage 0.18.3 ``ransac`` + ``EuclideanTransform`` (SVD Umeyama); this is the
  reference's CPU cost structure and is what ``bench.py`` times as cpu_baseline.
* ``filter_matches``: VA:196-214 (best-match reorder, ratio filter, median
  displacement filter, surviving template-index set) written with the same numpy
  calls as the reference.
* ``consensus`` / ``lookup``: VA:224-286 with real CPython ``set``/``Counter``.

Pinning: the RANSAC/consensus/filter restatements are checked against fixtures
made by running the reference's own code (tests/golden/make_golden.py); knnMatch
and warpAffine are pinned only by hand-computed known-answer tests because
OpenCV is absent from this image ("parity vs real OpenCV unpinned").
"""
from __future__ import annotations

import ctypes
import math
import os
from collections import Counter
from typing import Dict, List, Sequence, Set, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib() -> ctypes.CDLL:
    """Load (building if needed) the oracle shared library."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libkcmc_oracle.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        i = ctypes.c_int
        L.kcmc_oracle_knn2_l2u8.argtypes = [P, i, P, i, i, P, P]
        L.kcmc_oracle_knn2_hamming.argtypes = [P, i, P, i, i, P, P]
        L.kcmc_oracle_warp_affine_u16.argtypes = [P, i, i, i, P, i, P, i, i]
        L.kcmc_oracle_invert_affine.argtypes = [P, P]
        L.kcmc_oracle_pairwise_sum.argtypes = [P, i]
        L.kcmc_oracle_pairwise_sum.restype = ctypes.c_double
        L.kcmc_oracle_ransac_rigid.argtypes = [P, P, i, P, i, ctypes.c_double, P, P, P, P]
        L.kcmc_oracle_knn2_l2f32.argtypes = [P, i, P, i, i, P, P]
        L.kcmc_oracle_orb_detect.argtypes = [P, i, i, i, i, ctypes.c_double, i, P, P, P, P]
        L.kcmc_oracle_fast_score.argtypes = [P, i, i, i]
        L.kcmc_oracle_harris.argtypes = [P, i, i, i, ctypes.c_double]
        L.kcmc_oracle_harris.restype = ctypes.c_double
        L.kcmc_oracle_orientation_bin.argtypes = [P, i, i, i, P]
        L.kcmc_oracle_ransac_model.argtypes = [i, P, P, i, P, i, ctypes.c_double, P, P, P, P]
        L.kcmc_oracle_warp_perspective_u16.argtypes = [P, i, i, i, P, i, P, i, i]
        L.kcmc_oracle_invert_perspective.argtypes = [P, P]
        L.kcmc_oracle_pyr_down_u8.argtypes = [P, i, i, P, i, i]
        L.kcmc_oracle_invert_perspective.restype = i
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------- K1
def knn2_hamming(query: np.ndarray, train: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """OpenCV ``BFMatcher(cv2.NORM_HAMMING).knnMatch(query, train, k=2)`` on binary (uint8)
    descriptors: the opt-in extension matcher (the reference itself uses NORM_L2, VA:194).
    Same outputs as ``knn2_l2u8`` with integer bit-count distances."""
    q = np.ascontiguousarray(query, dtype=np.uint8)
    t = np.ascontiguousarray(train, dtype=np.uint8)
    assert q.ndim == 2 and t.ndim == 2 and q.shape[1] == t.shape[1]
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.float32)
    rc = lib().kcmc_oracle_knn2_hamming(_p(q), q.shape[0], _p(t), t.shape[0], q.shape[1], _p(idx), _p(dist))
    assert rc == 0
    return idx, dist


def knn2_l2u8(query: np.ndarray, train: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """OpenCV ``BFMatcher().knnMatch(query, train, k=2)`` for uint8 descriptors.

    Returns ``idx [n_query, 2]`` (train indices, -1 if absent) and
    ``dist [n_query, 2]`` float32 (FLT_MAX if absent).  VA:194-195 calls it with
    query = template descriptors, train = frame descriptors.
    """
    q = np.ascontiguousarray(query, dtype=np.uint8)
    t = np.ascontiguousarray(train, dtype=np.uint8)
    assert q.ndim == 2 and t.ndim == 2 and q.shape[1] == t.shape[1]
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.float32)
    rc = lib().kcmc_oracle_knn2_l2u8(_p(q), q.shape[0], _p(t), t.shape[0], q.shape[1], _p(idx), _p(dist))
    assert rc == 0
    return idx, dist


def knn2_l2f32(query: np.ndarray, train: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """``BFMatcher(NORM_L2).knnMatch(query, train, k=2)`` for float32 descriptors with
    the build's distance definition (sequential fp64 sum of squared differences,
    sqrtf of its float rounding; ties to the lower train index)."""
    q = np.ascontiguousarray(query, dtype=np.float32)
    t = np.ascontiguousarray(train, dtype=np.float32)
    assert q.ndim == 2 and t.ndim == 2 and q.shape[1] == t.shape[1]
    idx = np.empty((q.shape[0], 2), np.int32)
    dist = np.empty((q.shape[0], 2), np.float32)
    rc = lib().kcmc_oracle_knn2_l2f32(_p(q), q.shape[0], _p(t), t.shape[0], q.shape[1], _p(idx), _p(dist))
    assert rc == 0
    return idx, dist


def filter_matches(
    idx: np.ndarray,
    dist: np.ndarray,
    kp_template: np.ndarray,
    kp_query: np.ndarray,
    ratio: float = 0.75,
) -> Tuple[Set[int], np.ndarray, Tuple[int, int, int, int]]:
    """VA:196-221 from knnMatch output, with the reference's own numpy calls.

    Returns (kp_idxs set, kp_query_ordered [n_tpl,2] f64, log counts
    (len(kp_query) after reorder, len(matches), n_ratio, n_dist)).
    """
    n_tpl = idx.shape[0]
    kp_query_ordered = np.zeros_like(kp_template)
    for i in range(n_tpl):
        kp_query_ordered[i] = kp_query[idx[i, 0]]
    feature = [i for i in range(n_tpl) if float(dist[i, 0]) < ratio * float(dist[i, 1])]
    kt = np.array([kp_template[i] for i in feature])
    kq = np.array([kp_query_ordered[i] for i in feature])
    if feature:
        d = np.linalg.norm(kt - kq, axis=1)
        (d_1, d_2) = (0.5, 2)
        keep = np.where((d_1 * np.median(d) <= d) * (d <= d_2 * np.median(d)))[0]
        dist_matches = [feature[k] for k in keep]
    else:
        dist_matches = []
    kp_idxs = set(dist_matches)
    return kp_idxs, kp_query_ordered, (len(kp_query_ordered), n_tpl, len(feature), len(dist_matches))


# --------------------------------------------------------------------- consensus
def consensus(kp_idxs_list: Sequence[Set[int]], n_kp_global: int, n_min: int = 5) -> Tuple[Set[int], tuple, tuple]:
    """VA:224-249 with real Counter/set.  Returns (set, ordered idxs, counts)."""
    counts = Counter([x for s in kp_idxs_list for x in s])
    votes = [x for x in counts.most_common(n_kp_global)]
    if len(votes) < n_min:
        raise RuntimeError("Too few keypoints found")
    idxs, rates = zip(*votes)
    return set(idxs), idxs, rates


def lookup(consensus_idxs: Set[int], kp_idxs_list: Sequence[Set[int]]) -> List[List[int]]:
    """VA:271-278: per-frame template-index list in CPython set order."""
    return [list(consensus_idxs.intersection(s)) for s in kp_idxs_list]


# --------------------------------------------------------------------------- K2
_HYP_CACHE: Dict[Tuple[int, int, int], np.ndarray] = {}


def hypothesis_table(n: int, trials: int = 1000, seed: int = 42, min_samples: int = 2) -> np.ndarray:
    """Sample indices skimage 0.18.3 uses for trial t (fit.py:791, 819-826)."""
    key = (n, trials, seed, min_samples)
    if key not in _HYP_CACHE:
        rs = np.random.RandomState(seed)
        _HYP_CACHE[key] = np.array(
            [rs.choice(n, min_samples, replace=False) for _ in range(trials)], dtype=np.int32
        )
    return _HYP_CACHE[key]


def ransac_rigid(src: np.ndarray, dst: np.ndarray, trials: int = 1000, thresh: float = 2.0, seed: int = 42):
    """Closed-form restatement of VA:309-316 (skimage ransac + EuclideanTransform).

    src = frame keypoints, dst = template keypoints.  Returns
    (params [2,3] (NaN if no model), inliers bool [N], best_trial, n_inliers).
    """
    src = np.ascontiguousarray(src, np.float64)
    dst = np.ascontiguousarray(dst, np.float64)
    n = src.shape[0]
    hyp = np.ascontiguousarray(hypothesis_table(n, trials, seed))
    params = np.empty((2, 3), np.float64)
    inl = np.zeros(max(n, 1), np.uint8)
    bt = np.zeros(1, np.int32)
    ni = np.zeros(1, np.int32)
    lib().kcmc_oracle_ransac_rigid(_p(src), _p(dst), n, _p(hyp), trials, float(thresh), _p(params), _p(inl), _p(bt), _p(ni))
    return params, inl[:n].astype(bool), int(bt[0]), int(ni[0])


def compute_euclidean_affine(kp_template, kp_query, spatial_downsample_rate=1, n_skip=3, **kw):
    """VA:288-323 on top of ``ransac_rigid``."""
    if len(kp_query) < n_skip:
        return np.full((2, 3), np.nan)
    params, _, _, _ = ransac_rigid(kp_query, kp_template, **kw)
    params = params.copy()
    params[:, 2] *= spatial_downsample_rate
    return params


def _umeyama_rigid_numpy(src, dst):
    """skimage _umeyama(src, dst, estimate_scale=False), _geometric.py:72-144."""
    num, dim = src.shape
    src_mean = src.mean(axis=0)
    dst_mean = dst.mean(axis=0)
    src_demean = src - src_mean
    dst_demean = dst - dst_mean
    A = dst_demean.T @ src_demean / num
    d = np.ones((dim,), dtype=np.double)
    if np.linalg.det(A) < 0:
        d[dim - 1] = -1
    T = np.eye(dim + 1, dtype=np.double)
    U, S, V = np.linalg.svd(A)
    rank = np.linalg.matrix_rank(A)
    if rank == 0:
        return np.nan * T
    if rank == dim - 1:
        if np.linalg.det(U) * np.linalg.det(V) > 0:
            T[:dim, :dim] = U @ V
        else:
            dd = d.copy()
            dd[dim - 1] = -1
            T[:dim, :dim] = U @ np.diag(dd) @ V
    else:
        T[:dim, :dim] = U @ np.diag(d) @ V
    T[:dim, dim] = dst_mean - (T[:dim, :dim] @ src_mean.T)
    return T


def _apply_rigid_numpy(T, coords):
    x, y = np.transpose(coords)
    s = np.vstack((x, y, np.ones_like(x)))
    d = s.T @ T.T
    d[d[:, 2] == 0, 2] = np.finfo(float).eps
    d[:, :2] /= d[:, 2:3]
    return d[:, :2]


def ransac_rigid_skimage(src, dst, trials=1000, thresh=2.0, seed=42):
    """Operation-for-operation numpy restatement of skimage 0.18.3 ransac with
    EuclideanTransform (fit.py:784-881); per-trial SVD like the reference.
    Slow by design: this is the reference CPU cost that bench.py reports."""
    rs = np.random.RandomState(seed)
    n = len(src)
    best_T, best_n, best_S, best_inl = None, 0, np.inf, None
    spl = rs.choice(n, 2, replace=False)
    for _ in range(trials):
        s_src, s_dst = src[spl], dst[spl]
        spl = rs.choice(n, 2, replace=False)
        T = _umeyama_rigid_numpy(s_src, s_dst)
        r = np.abs(np.sqrt(np.sum((_apply_rigid_numpy(T, src) - dst) ** 2, axis=1)))
        inl = r < thresh
        S = np.sum(r ** 2)
        ni = np.sum(inl)
        if ni > best_n or (ni == best_n and S < best_S):
            best_T, best_n, best_S, best_inl = T, ni, S, inl
            if best_S <= 0:
                break
    if best_inl is not None and any(best_inl):
        best_T = _umeyama_rigid_numpy(src[best_inl], dst[best_inl])
        return best_T[:2], best_inl
    return np.full((2, 3), np.nan), None


# ------------------------------------------------- K2 extension: affine / projective
MODEL_IDS = {"affine": 1, "projective": 2}
MODEL_MIN_SAMPLES = {"affine": 3, "projective": 4}
_TLS_COEFFS = {"affine": list(range(6)), "projective": list(range(8))}


def _center_and_normalize(points: np.ndarray):
    """skimage 0.18.3 _center_and_normalize_points (_geometric.py:18-69), restated:
    the Hartley similarity taking the centroid to 0 and the rms distance to sqrt(2).
    Raises ZeroDivisionError for coincident points, like skimage."""
    centroid = np.mean(points, axis=0)
    rms = math.sqrt(np.sum((points - centroid) ** 2) / points.shape[0])
    nf = math.sqrt(2) / rms
    N = np.array([[nf, 0, -nf * centroid[0]], [0, nf, -nf * centroid[1]], [0, 0, 1]])
    ph = np.vstack([points.T, np.ones(points.shape[0])])
    q = (N @ ph).T
    out = q[:, :2]
    out[:, 0] /= q[:, 2]
    out[:, 1] /= q[:, 2]
    return N, out


def estimate_tls(src: np.ndarray, dst: np.ndarray, model: str):
    """ProjectiveTransform/AffineTransform.estimate of skimage 0.18.3
    (_geometric.py:596-703): total least squares through np.linalg.svd of the 2N x 7
    (affine) / 2N x 9 (projective) system in Hartley-normalised coordinates.
    Returns (ok, params); params is NaN on ZeroDivisionError and None when
    np.isclose(V[-1,-1], 0) (skimage then leaves the previous params in place)."""
    try:
        Ns, s = _center_and_normalize(np.asarray(src, np.float64))
        Nd, d = _center_and_normalize(np.asarray(dst, np.float64))
    except ZeroDivisionError:
        return False, np.full((3, 3), np.nan)
    xs, ys, xd, yd = s[:, 0], s[:, 1], d[:, 0], d[:, 1]
    n = s.shape[0]
    A = np.zeros((2 * n, 9))
    A[:n, 0], A[:n, 1], A[:n, 2] = xs, ys, 1
    A[n:, 3], A[n:, 4], A[n:, 5] = xs, ys, 1
    A[:n, 6], A[:n, 7], A[:n, 8] = -xd * xs, -xd * ys, xd
    A[n:, 6], A[n:, 7], A[n:, 8] = -yd * xs, -yd * ys, yd
    cols = _TLS_COEFFS[model] + [8]
    _, _, V = np.linalg.svd(A[:, cols])
    if np.isclose(V[-1, -1], 0):
        return False, None
    H = np.zeros((3, 3))
    H.flat[_TLS_COEFFS[model]] = -V[-1, :-1] / V[-1, -1]
    H[2, 2] = 1
    return True, np.linalg.inv(Nd) @ H @ Ns


def _apply_h(H: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """ProjectiveTransform._apply_mat (_geometric.py:548-562)."""
    x, y = np.transpose(pts)
    q = np.vstack((x, y, np.ones_like(x))).T @ H.T
    q[q[:, 2] == 0, 2] = np.finfo(float).eps
    q[:, :2] /= q[:, 2:3]
    return q[:, :2]


def ransac_model(src, dst, model: str, trials: int = 1000, thresh: float = 2.0, seed: int = 42):
    """skimage ransac(..., AffineTransform/ProjectiveTransform, min_samples=3/4, ...)
    with the hypothesis loop in closed form (C) and skimage's own SVD refit on the
    inliers.  src = frame keypoints, dst = template keypoints.  Returns (params [3,3]
    (NaN if no model), inliers bool [N], best_trial, n_inliers)."""
    src = np.ascontiguousarray(src, np.float64)
    dst = np.ascontiguousarray(dst, np.float64)
    n = src.shape[0]
    ms = MODEL_MIN_SAMPLES[model]
    hyp = np.ascontiguousarray(hypothesis_table(n, trials, seed, ms))
    hm = np.empty(9, np.float64)
    inl = np.zeros(max(n, 1), np.uint8)
    bt = np.zeros(1, np.int32)
    ni = np.zeros(1, np.int32)
    rc = lib().kcmc_oracle_ransac_model(MODEL_IDS[model], _p(src), _p(dst), n, _p(hyp), trials, float(thresh),
                                        _p(hm), _p(inl), _p(bt), _p(ni))
    assert rc in (0, 1), rc
    inliers = inl[:n].astype(bool)
    if rc == 1:
        return np.full((3, 3), np.nan), inliers, int(bt[0]), int(ni[0])
    ok, H = estimate_tls(src[inliers], dst[inliers], model)
    if H is None:  # refit degenerate: skimage keeps the hypothesis model
        H = hm.reshape(3, 3).copy()
    return H, inliers, int(bt[0]), int(ni[0])


def ransac_model_skimage(src, dst, model: str, trials: int = 1000, thresh: float = 2.0, seed: int = 42):
    """Operation-for-operation numpy restatement of skimage 0.18.3 ransac with
    AffineTransform / ProjectiveTransform (fit.py:784-881; one SVD per trial).  Slow by
    design: the reference-style CPU cost structure.  Returns (params [3,3], inliers)."""
    rs = np.random.RandomState(seed)
    n = len(src)
    ms = MODEL_MIN_SAMPLES[model]
    best_H, best_n, best_S, best_inl = None, 0, np.inf, None
    spl = rs.choice(n, ms, replace=False)
    for _ in range(trials):
        s_src, s_dst = src[spl], dst[spl]
        spl = rs.choice(n, ms, replace=False)
        ok, H = estimate_tls(s_src, s_dst, model)
        if not ok:
            continue
        r = np.abs(np.sqrt(np.sum((_apply_h(H, src) - dst) ** 2, axis=1)))
        inl = r < thresh
        S = np.sum(r ** 2)
        ni = np.sum(inl)
        if ni > best_n or (ni == best_n and S < best_S):
            best_H, best_n, best_S, best_inl = H, ni, S, inl
            if best_S <= 0:
                break
    if best_inl is not None and any(best_inl):
        ok, H = estimate_tls(src[best_inl], dst[best_inl], model)
        return (best_H if H is None else H), best_inl
    return np.full((3, 3), np.nan), None


# --------------------------------------------------------------------------- K3
def invert_affine(M: np.ndarray) -> np.ndarray:
    M = np.ascontiguousarray(M, np.float64).reshape(6)
    out = np.empty(6, np.float64)
    lib().kcmc_oracle_invert_affine(_p(M), _p(out))
    return out.reshape(2, 3)


def pyr_down_u8(img: np.ndarray, dstsize=None) -> np.ndarray:
    """``cv2.pyrDown(img, dstsize=dstsize)`` on a uint8 [H, W] frame (VA:501-503).

    ``dstsize`` is (width, height) like OpenCV; empty/None -> ((W+1)//2, (H+1)//2).
    Raises ValueError where OpenCV's size assertion fails.
    """
    src = np.ascontiguousarray(img, np.uint8)
    H, W = src.shape
    dW, dH = ((W + 1) // 2, (H + 1) // 2) if dstsize is None or min(dstsize) <= 0 else dstsize
    out = np.empty((dH, dW), np.uint8)
    if lib().kcmc_oracle_pyr_down_u8(_p(src), H, W, _p(out), int(dH), int(dW)) != 0:
        raise ValueError("pyrDown: std::abs(dsize.width*2 - ssize.width) <= 2 && "
                         "std::abs(dsize.height*2 - ssize.height) <= 2")
    return out


def warp_affine_u16(img: np.ndarray, M: np.ndarray, dsize=None, inverse_map: bool = False) -> np.ndarray:
    """OpenCV ``warpAffine(img, M, dsize, INTER_LINEAR)`` on uint16, border 0.

    ``img`` is [H,W] or [H,W,C]; ``dsize`` is (W, H) like OpenCV (default: same).
    """
    src = np.ascontiguousarray(img, np.uint16)
    H, W = src.shape[:2]
    C = 1 if src.ndim == 2 else src.shape[2]
    dW, dH = (W, H) if dsize is None else dsize
    out = np.empty((dH, dW) + (() if src.ndim == 2 else (C,)), np.uint16)
    M6 = np.ascontiguousarray(M, np.float64).reshape(6)
    rc = lib().kcmc_oracle_warp_affine_u16(_p(src), H, W, C, _p(M6), int(inverse_map), _p(out), dH, dW)
    assert rc == 0
    return out


def pairwise_sum(a: np.ndarray) -> float:
    a = np.ascontiguousarray(a, np.float64)
    return lib().kcmc_oracle_pairwise_sum(_p(a), a.size)


# ------------------------------------------------------------ K3 extension: perspective
def invert_perspective(M: np.ndarray) -> np.ndarray:
    """cv::invert of a 3x3 double matrix (OpenCV's closed-form 3x3 branch)."""
    M9 = np.ascontiguousarray(M, np.float64).reshape(9)
    out = np.empty(9, np.float64)
    lib().kcmc_oracle_invert_perspective(_p(M9), _p(out))
    return out.reshape(3, 3)


def warp_perspective_u16(img: np.ndarray, M: np.ndarray, dsize=None, inverse_map: bool = False) -> np.ndarray:
    """OpenCV ``warpPerspective(img, M, dsize, INTER_LINEAR)`` on uint16, border 0
    (classic WarpPerspectiveInvoker + remapBilinear arithmetic)."""
    src = np.ascontiguousarray(img, np.uint16)
    H, W = src.shape[:2]
    C = 1 if src.ndim == 2 else src.shape[2]
    dW, dH = (W, H) if dsize is None else dsize
    out = np.empty((dH, dW) + (() if src.ndim == 2 else (C,)), np.uint16)
    M9 = np.ascontiguousarray(M, np.float64).reshape(9)
    rc = lib().kcmc_oracle_warp_perspective_u16(_p(src), H, W, C, _p(M9), int(inverse_map), _p(out), dH, dW)
    assert rc == 0
    return out


# ------------------------------------------------------------ f1: detection
def orb_detect(img: np.ndarray, n_features: int = 500, threshold: int = 20, harris_k: float = 0.04, edge: int = 16,
               pattern: np.ndarray = None, bin_cs: np.ndarray = None):
    """The build's ORB-style detector on one uint8 image (kcmc_oracle_orb_detect):
    returns (kp [n, 2] f64 (x, y), des [n, 32] u8) in candidate order."""
    a = np.ascontiguousarray(img, np.uint8)
    H, W = a.shape
    pat = np.ascontiguousarray(pattern, np.int8)
    cs = np.ascontiguousarray(bin_cs, np.float64)
    kp = np.empty((max(n_features, 1), 2), np.float64)
    des = np.empty((max(n_features, 1), 32), np.uint8)
    n = lib().kcmc_oracle_orb_detect(_p(a), H, W, threshold, n_features, float(harris_k), edge, _p(pat), _p(cs),
                                     _p(kp), _p(des))
    assert n >= 0
    return kp[:n].copy(), des[:n].copy()
