"""Seeded random sweeps of the hot-path kernels against the CPU oracle: shapes, channel
counts, value ranges, map families and descriptor layouts drawn at random (fixed seeds,
so a failure names its case and reproduces).  Every output is compared bit for bit.

Warp (VA:455-458): frame sizes 1 x 1 to 300 x 520 (odd, partial tiles,
W % 8 != 0), C = 1 / 3 / 4, values 14-bit / full / hot pixels, maps from near-identity to
40-degree rotations, anisotropic zoom and shear, shifts off the frame, forward and inverse,
affine and perspective (mild, strong, and denominators that change sign over the frame).
Matchers (VA:194-195): u8 L2 and Hamming over D = 1..64 and float32 over D = 1..128, with
exact copies of template rows (ties resolved by the lower frame index) and frames of 2 rows.
"""
import numpy as np
import pytest
import torch

import oracle
from kcmc_amd import stages

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _values(rng, shape):
    kind = rng.integers(0, 3)
    if kind == 0:
        v = rng.integers(0, 16384, shape)
    elif kind == 1:
        v = rng.integers(0, 65536, shape)
    else:
        v = rng.integers(0, 8192, shape)
        v[rng.random(shape) < 1e-3] = 65535
    return v.astype(np.uint16)


def _affine(rng, H, W):
    fam = rng.integers(0, 5)
    if fam == 0:  # near identity
        a, s, sh = rng.normal(0, 0.01), 1.0, 0.0
        t = rng.normal(0, 3, 2)
    elif fam == 1:  # large rotation
        a, s, sh = rng.uniform(-0.7, 0.7), 1.0, 0.0
        t = rng.normal(0, W / 4, 2)
    elif fam == 2:  # zoom / anisotropic scale with shear
        a, s, sh = rng.normal(0, 0.05), rng.uniform(0.5, 2.0), rng.normal(0, 0.1)
        t = rng.normal(0, 10, 2)
    elif fam == 3:  # far off the frame
        a, s, sh = 0.0, 1.0, 0.0
        t = np.array([rng.choice([-1, 1]) * (W + rng.uniform(5, 50)), 0.0])
    else:  # small rotation, sub-pixel shift
        a, s, sh = rng.normal(0, 0.03), 1.0, 0.0
        t = rng.uniform(-2, 2, 2)
    c, n = np.cos(a), np.sin(a)
    sy = s * rng.uniform(0.9, 1.1)
    return np.array([[s * c, -n + sh, t[0]], [n, sy * c, t[1]]])


def _perspective(rng, H, W):
    M = np.vstack([_affine(rng, H, W), [0.0, 0.0, 1.0]])
    fam = rng.integers(0, 3)
    if fam == 0:
        M[2, :2] = rng.normal(0, 2e-5, 2)
    elif fam == 1:
        M[2, :2] = rng.normal(0, 5e-4, 2)
    else:  # the denominator changes sign inside the frame: direct gather / zeros
        M[2, :2] = [2.0 / max(W, 1), -1.0 / max(H, 1)]
    return M


@pytest.mark.parametrize("seed", range(24))
def test_warp_fuzz_vs_oracle(dev, seed):
    rng = np.random.default_rng(1000 + seed)
    F = int(rng.integers(1, 4))
    H, W = int(rng.integers(1, 301)), int(rng.integers(1, 521))
    if seed % 6 == 0:
        W = 8 * int(rng.integers(1, 65))  # the vector-staged paths (W % 8 == 0)
    C = int(rng.choice([1, 1, 3, 4]))
    shape = (F, H, W) if C == 1 else (F, H, W, C)
    imgs = _values(rng, shape)
    persp = bool(seed % 2)
    Ms = np.stack([(_perspective if persp else _affine)(rng, H, W) for _ in range(F)])
    inv = bool(rng.integers(0, 2))
    fn = stages.warp_perspective_u16 if persp else stages.warp_affine_u16
    ref = oracle.warp_perspective_u16 if persp else oracle.warp_affine_u16
    out = fn(_t(imgs, dev), _t(Ms, dev), inverse_map=inv).cpu().numpy()
    for f in range(F):
        exp = ref(imgs[f], Ms[f], inverse_map=inv)
        assert np.array_equal(out[f], exp), (seed, f, shape, persp, inv, int((out[f] != exp).sum()))


def _frames_with_ties(rng, tpl, n_frames, max_rows, gen):
    frames = []
    for _ in range(n_frames):
        n_q = int(rng.choice([2, 3, int(rng.integers(2, max_rows + 1))]))
        q = gen(n_q)
        k = n_q // 4
        if k:
            q[:k] = tpl[rng.integers(0, tpl.shape[0], k)]  # exact copies: distance 0 ties
        if n_q > 6:
            q[5] = q[1]  # duplicate frame rows: equal distances, the lower index wins
        frames.append(q)
    return frames


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("kind", ["l2u8", "hamming", "l2f32"])
def test_knn2_fuzz_vs_oracle(dev, kind, seed):
    rng = np.random.default_rng(2000 + 17 * seed + len(kind))
    if kind == "l2f32":
        D = int(rng.integers(1, 129))
        gen = lambda n: rng.normal(0, rng.choice([1e-3, 1.0, 50.0]), (n, D)).astype(np.float32)  # noqa: E731
    else:
        D = int(rng.integers(1, 65))
        gen = lambda n: rng.integers(0, 256, (n, D), dtype=np.uint8)  # noqa: E731
    n_tpl = int(rng.integers(1, 700))
    tpl = gen(n_tpl)
    frames = _frames_with_ties(rng, tpl, int(rng.integers(1, 6)), 900, gen)
    off = np.zeros(len(frames) + 1, np.int32)
    off[1:] = np.cumsum([len(q) for q in frames])
    des_q = np.concatenate(frames)
    if kind == "hamming":
        idx, dist = stages.knn2_hamming(_t(tpl, dev), _t(des_q, dev), _t(off, dev), int(np.diff(off).max()))
        ora = oracle.knn2_hamming
    else:
        idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(des_q, dev), _t(off, dev), int(np.diff(off).max()))
        ora = oracle.knn2_l2f32 if kind == "l2f32" else oracle.knn2_l2u8
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = ora(tpl, q)
        assert np.array_equal(idx[f], ri), (seed, kind, f, D, n_tpl, len(q))
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), (seed, kind, f)


def _csr(lists):
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    return off


def _point_sets(rng, n_frames, model):
    """Frame / template point pairs: random sizes (including 0-3 points), coordinate
    scales from 1e-2 to 1e4, noise from exact to large, outlier shares, duplicated pairs."""
    tpls, qs = [], []
    for _ in range(n_frames):
        N = int(rng.choice([0, 1, 2, 3, 4, 5, int(rng.integers(6, 60)), int(rng.integers(60, 400))]))
        scale = 10.0 ** rng.uniform(-2, 4)
        tpl = rng.uniform(0, scale, (N, 2))
        a = rng.normal(0, 0.05)
        A = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
        if model != "rigid":
            A = A @ np.array([[rng.uniform(0.8, 1.25), rng.normal(0, 0.05)], [0.0, rng.uniform(0.8, 1.25)]])
        q = tpl @ A.T + rng.normal(0, scale * 0.01, 2)
        noise = rng.choice([0.0, 1e-9, 0.3, 1.5]) * (scale / 1000.0 if scale > 1000 else 1.0)
        q = q + rng.normal(0, noise, (N, 2)) if noise else q
        out = rng.random(N) < rng.uniform(0, 0.5)
        q[out] = rng.uniform(0, scale, (int(out.sum()), 2))
        if N > 10 and rng.random() < 0.3:
            q[N // 2:], tpl[N // 2:] = q[: N - N // 2], tpl[: N - N // 2]
        tpls.append(tpl)
        qs.append(q)
    return tpls, qs


@pytest.mark.parametrize("seed", range(6))
def test_ransac_rigid_fuzz_vs_oracle(dev, seed):
    rng = np.random.default_rng(3000 + seed)
    tpls, qs = _point_sets(rng, 24, "rigid")
    thresh = float(rng.choice([2.0, 0.5, 5.0, 1e-3]))
    off = _csr(qs)
    r = stages.ransac_rigid(_t(np.concatenate(qs).reshape(-1, 2), dev), _t(np.concatenate(tpls).reshape(-1, 2), dev),
                            _t(off, dev), off, residual_threshold=thresh)
    params, inl = r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool)
    nin, best = r.n_inliers.cpu().numpy(), r.best_trial.cpu().numpy()
    for f in range(len(qs)):
        if len(qs[f]) < 3:  # N_KP_FRAME_SKIP: no model, NaN (VA:307)
            assert np.isnan(params[f]).all(), (seed, f)
            continue
        p, i_ref, bt, ni = oracle.ransac_rigid(qs[f], tpls[f], thresh=thresh)
        assert best[f] == bt and nin[f] == ni, (seed, f, len(qs[f]))
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), (seed, f)
        np.testing.assert_allclose(params[f], p, rtol=1e-10, atol=1e-10 * max(1.0, np.abs(tpls[f]).max()),
                                   equal_nan=True, err_msg=str((seed, f)))


@pytest.mark.parametrize("model", ["rigid", "affine", "projective"])
@pytest.mark.parametrize("scale", [1.0, 2000.0, 3e5])
def test_ransac_threshold_band_vs_oracle(dev, model, scale):
    """Points whose residual under the true map lies within 1e-12 .. 1e-2 of the threshold
    (2 px), so the fp32 phase A (ransac_common.h score32) must leave them undecided and the
    trials that reach the best count are counted again in fp64 (phase A2): counts, inliers,
    winning trial bit-exact, params as the oracle.  Coordinates up to 3e5 px make the fp32
    band wide (and past ~1e5 px the trials fall back to the fp64 phase A)."""
    rng = np.random.default_rng(int(scale) + {"rigid": 0, "affine": 1, "projective": 2}[model])
    tpls, qs = [], []
    for f in range(6):
        n_exact, n_band, n_out = 12 + 3 * f, 20, 10
        tpl = rng.uniform(0.2, 1.0, (n_exact + n_band + n_out, 2)) * scale
        a = rng.normal(0, 0.02)
        A = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
        if model != "rigid":
            A = A @ np.array([[1.01, 0.02], [0.0, 0.99]])
        t = rng.normal(0, 5, 2)
        q = (tpl - t) @ np.linalg.inv(A).T  # q maps onto tpl exactly: A q + t = tpl
        # band points: displace the template point by 2 + d px along a random direction
        d = rng.choice([-1e-2, -1e-5, -1e-9, -1e-12, 0.0, 1e-12, 1e-9, 1e-5, 1e-2], n_band)
        ang = rng.uniform(0, 2 * np.pi, n_band)
        sl = slice(n_exact, n_exact + n_band)
        tpl[sl] += (2.0 + d)[:, None] * np.stack([np.cos(ang), np.sin(ang)], 1)
        tpl[n_exact + n_band:] += rng.uniform(5, 50, (n_out, 2))
        tpls.append(tpl)
        qs.append(q)
    off = _csr(qs)
    args = (_t(np.concatenate(qs), dev), _t(np.concatenate(tpls), dev), _t(off, dev), off)
    r = stages.ransac_rigid(*args) if model == "rigid" else stages.ransac_model(*args, model=model)
    params, inl = r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool)
    nin, best = r.n_inliers.cpu().numpy(), r.best_trial.cpu().numpy()
    for f in range(len(qs)):
        if model == "rigid":
            p, i_ref, bt, ni = oracle.ransac_rigid(qs[f], tpls[f])
        else:
            p, i_ref, bt, ni = oracle.ransac_model(qs[f], tpls[f], model)
        assert best[f] == bt and nin[f] == ni, (model, scale, f, best[f], bt, nin[f], ni)
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), (model, scale, f)
        if model == "rigid":
            np.testing.assert_allclose(params[f], p, rtol=1e-10, atol=1e-10 * scale)
        else:
            _check_refit(params[f], p, qs[f][i_ref], tpls[f][i_ref], model, ni, (model, scale, f))


def _tls_model(A, Ns, Nd, model, v):
    H = np.zeros((3, 3))
    cols = [0, 1, 2, 3, 4, 5] if model == "affine" else list(range(8))
    H.flat[cols] = -v[:-1] / v[-1]
    H[2, 2] = 1
    return np.linalg.inv(Nd) @ H @ Ns


def _tls_spread(src, dst, model, sc):
    """How far LAPACK's own answers to the refit's total-least-squares problem spread
    (skimage: np.linalg.svd of the normalised 2N x 7 / 2N x 9 system, _geometric.py:596-703):
    the gesvd driver, and gesdd on the rows mixed by a random orthogonal matrix (the same
    problem, rounded differently), in the metric the comparison uses:
    max |dH| / (|H| + 0.1 max(1, sc)).  About 1e-12 on every fuzz case
    (tools/debug/refit_spread.py); the comparison's tolerance is max(1e-8, 100 x this)."""
    import scipy.linalg

    Ns, s = oracle._center_and_normalize(np.asarray(src, np.float64))
    Nd, d = oracle._center_and_normalize(np.asarray(dst, np.float64))
    n = len(s)
    A = np.zeros((2 * n, 9))
    A[:n, 0:2], A[:n, 2], A[n:, 3:5], A[n:, 5] = s, 1, s, 1
    A[:n, 6:8], A[:n, 8] = -s * d[:, :1], d[:, 0]
    A[n:, 6:8], A[n:, 8] = -s * d[:, 1:2], d[:, 1]
    if model == "affine":
        A = A[:, [0, 1, 2, 3, 4, 5, 8]]
    ref = _tls_model(A, Ns, Nd, model, np.linalg.svd(A)[2][-1])
    Q, _ = np.linalg.qr(np.random.default_rng(0).normal(size=(len(A), len(A))))
    alts = [scipy.linalg.svd(A, lapack_driver="gesvd")[2][-1], np.linalg.svd(Q @ A)[2][-1]]
    return max(float(np.max(np.abs(_tls_model(A, Ns, Nd, model, v) - ref) / (np.abs(ref) + 0.1 * max(1.0, sc))))
               for v in alts)


def _check_refit(params, p, src, dst, model, ni, ctx):
    """The refit vs skimage's (north_star: parameters within 1e-4 relative): per entry
    |dH| <= r (|H| + 0.1 max(1, |dst|)) with r = max(1e-8, 100 x LAPACK's own spread on the
    problem) -- no case is skipped."""
    sc = float(np.abs(dst).max()) if len(dst) else 1.0
    ms = 3 if model == "affine" else 4
    r = 1e-8
    if ni >= ms and np.isfinite(p).all():
        try:
            r = max(r, 100.0 * _tls_spread(src, dst, model, sc))
        except (ZeroDivisionError, np.linalg.LinAlgError):
            pass
    assert r <= 1e-4, (ctx, r)  # the problem determines the model to north_star's tolerance
    np.testing.assert_allclose(params, p, rtol=r, atol=0.1 * max(1.0, sc) * r, equal_nan=True, err_msg=str(ctx))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("model", ["affine", "projective"])
def test_ransac_model_fuzz_vs_oracle(dev, model, seed):
    rng = np.random.default_rng(4000 + seed + (100 if model == "projective" else 0))
    tpls, qs = _point_sets(rng, 12, model)
    ms = 3 if model == "affine" else 4
    for f in range(len(qs)):  # n_skip <= N <= min_samples raises ValueError, as skimage does
        if 3 <= len(qs[f]) <= ms:
            tpls[f], qs[f] = tpls[f][:2], qs[f][:2]
    off = _csr(qs)
    r = stages.ransac_model(_t(np.concatenate(qs).reshape(-1, 2), dev), _t(np.concatenate(tpls).reshape(-1, 2), dev),
                            _t(off, dev), off, model=model)
    params, inl = r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool)
    nin, best = r.n_inliers.cpu().numpy(), r.best_trial.cpu().numpy()
    for f in range(len(qs)):
        if len(qs[f]) < 3:
            assert np.isnan(params[f]).all(), (seed, f)
            continue
        p, i_ref, bt, ni = oracle.ransac_model(qs[f], tpls[f], model)
        assert best[f] == bt and nin[f] == ni, (seed, f, len(qs[f]))
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), (seed, f)
        _check_refit(params[f], p, qs[f][i_ref], tpls[f][i_ref], model, ni, (seed, f))


@pytest.mark.parametrize("model,seed,frame", [("projective", 20410, 3), ("affine", 20428, 11), ("affine", 20316, 7),
                                              ("projective", 20328, 0), ("projective", 20371, 3)])
def test_ransac_model_refit_hard_cases(dev, model, seed, frame):
    """Refits the round-5 solver (inverse iteration on A^T A) missed: seed 20410 frame 3, a
    homography from 4 inliers whose TLS vector's last component is 1.2e-5 of its norm
    (entries up to 2.7e8; the round-5 GPU refit was 1.3e-3 off), and seed 20428 frame 11,
    397 affine inliers whose two smallest singular values differ by 0.16 % (inverse iteration
    stalls; LAPACK's drivers agree to 1e-15)."""
    rng = np.random.default_rng(4000 + seed + (100 if model == "projective" else 0))
    tpls, qs = _point_sets(rng, 12, model)
    ms = 3 if model == "affine" else 4
    for f in range(len(qs)):
        if 3 <= len(qs[f]) <= ms:
            tpls[f], qs[f] = tpls[f][:2], qs[f][:2]
    q, t = qs[frame], tpls[frame]
    off = np.array([0, len(q)], np.int32)
    r = stages.ransac_model(_t(q, dev), _t(t, dev), _t(off, dev), off, model=model)
    p, i_ref, bt, ni = oracle.ransac_model(q, t, model)
    assert int(r.best_trial[0]) == bt and int(r.n_inliers[0]) == ni
    assert np.array_equal(r.inliers.cpu().numpy().astype(bool), i_ref)
    _check_refit(r.params[0].cpu().numpy(), p, q[i_ref], t[i_ref], model, ni, (model, seed, frame))


@pytest.mark.parametrize("seed", range(8))
def test_match_filters_fuzz_vs_oracle(dev, seed):
    """VA:196-221 on random knn results (kcmc_match_filter): ratio-test boundaries
    (d0 == 0.75 d1 in float, equal distances, zeros), displacement medians with exact
    boundary values, template counts on all three filter kernels (<= 512, <= 4096, more)."""
    rng = np.random.default_rng(5000 + seed)
    n_tpl = int(rng.choice([1, 2, 7, 100, 512, 513, 2000, 4096, 5000, 8192]))
    F = int(rng.integers(1, 5))
    q_lists = [rng.uniform(0, 500, (int(rng.integers(2, 300)), 2)) for _ in range(F)]
    kp_tpl = rng.uniform(0, 500, (n_tpl, 2))
    idx = np.zeros((F, n_tpl, 2), np.int32)
    dist = np.zeros((F, n_tpl, 2), np.float32)
    for f, q in enumerate(q_lists):
        idx[f] = rng.integers(0, len(q), (n_tpl, 2))
        d1 = rng.uniform(0, 300, n_tpl).astype(np.float32)
        d0 = (d1 * rng.uniform(0, 1, n_tpl)).astype(np.float32)
        k = rng.random(n_tpl)
        d0[k < 0.1] = (np.float32(0.75) * d1[k < 0.1]).astype(np.float32)  # on the ratio boundary
        d0[(k >= 0.1) & (k < 0.15)] = d1[(k >= 0.1) & (k < 0.15)]
        d0[(k >= 0.15) & (k < 0.18)] = 0
        dist[f, :, 0], dist[f, :, 1] = d0, d1
        if n_tpl > 4:  # a few template points displaced exactly onto the 0.5x / 2x median boundaries
            kp_tpl[:2] = q[idx[f, :2, 0]]
    off = _csr(q_lists)
    kq = np.concatenate(q_lists)
    res = stages.filter_matches((_t(idx, dev), _t(dist, dev)), _t(kp_tpl, dev), _t(kq, dev), _t(off, dev))
    bits = res.keep_bits.cpu().numpy().view(np.uint32)
    kqo, cnt = res.kp_ordered.cpu().numpy(), res.counts.cpu().numpy()
    for f, q in enumerate(q_lists):
        s, kq_ref, c = oracle.filter_matches(idx[f], dist[f], kp_tpl, q)
        kept = [i for i in range(n_tpl) if (bits[f, i >> 5] >> (i & 31)) & 1]
        assert kept == sorted(s), (seed, f, n_tpl)
        assert np.array_equal(kqo[f], kq_ref), (seed, f)
        assert cnt[f].tolist() == list(c), (seed, f)


@pytest.mark.parametrize("seed", range(8))
def test_slab_end_to_end_fuzz_vs_oracle(dev, seed):
    """align_slab on random slabs (frame count, size, channels, template size, descriptor
    kind and length, RANSAC model, consensus size) against the oracle stage by stage
    (test_gpu_configs._check_slab: match + filters on every frame, CPython-ordered
    consensus, RANSAC on every frame, the warp of every frame bit-exact)."""
    from test_gpu_configs import _check_slab

    rng = np.random.default_rng(6000 + seed)
    descriptor = str(rng.choice(["u8", "u8", "f32"]))
    D = int(rng.integers(16, 65)) if descriptor == "u8" else int(rng.integers(16, 129))
    _check_slab(dev, F=int(rng.integers(2, 25)), H=int(rng.integers(64, 301)), W=int(rng.integers(64, 401)),
                C=int(rng.choice([1, 1, 3, 4])), n_tpl=int(rng.integers(40, 600)), D=D,
                model=str(rng.choice(["euclidean", "affine", "projective"])),
                n_kp_global=int(rng.integers(10, 120)), descriptor=descriptor, seed=7000 + seed)


@pytest.mark.parametrize("seed", range(10))
def test_pyr_down_and_normalize_fuzz(dev, seed):
    """pyrDown (VA:501-503) at random sizes and every admissible dstsize, and the
    99.99th-percentile max-scale (VA:479-492) of random uint16 stacks (numpy's own
    percentile and clip as the reference writes them) -- bit for bit."""
    rng = np.random.default_rng(8000 + seed)
    F, H, W = int(rng.integers(1, 4)), int(rng.integers(1, 260)), int(rng.integers(1, 400))
    imgs = rng.integers(0, 256, (F, H, W)).astype(np.uint8)
    sizes = [((W + 1) // 2, (H + 1) // 2)] + [(dw, dh) for dw in (W // 2, (W + 2) // 2) for dh in (H // 2, (H + 2) // 2)
                                             if dw >= 1 and dh >= 1 and abs(2 * dw - W) <= 2 and abs(2 * dh - H) <= 2]
    for dw, dh in sorted(set(sizes)):
        out = stages.pyr_down_u8(_t(imgs, dev), (dw, dh)).cpu().numpy()
        for f in range(F):
            assert np.array_equal(out[f], oracle.pyr_down_u8(imgs[f], (dw, dh))), (seed, f, (H, W), (dw, dh))
    hi = int(rng.choice([255, 4095, 16383, 65535]))
    x = rng.integers(0, hi + 1, (F, H, W)).astype(np.uint16)
    if rng.random() < 0.5:  # a few saturated / hot pixels above the bulk
        x[rng.random(x.shape) < 1e-4] = 65535
    b = stages.brightest_px(_t(x, dev))
    assert b == np.percentile(x, 99.99), (seed, b)
    if b > 0:
        got = stages.max_scale_u8(_t(x, dev), b).cpu().numpy()
        assert np.array_equal(got, np.clip(x / b * 255, a_min=0, a_max=255).astype(np.uint8)), seed


@pytest.mark.parametrize("seed", range(6))
def test_orb_detect_fuzz_vs_oracle(dev, seed):
    """The build-defined GPU ORB detector (f1) against its C restatement on random
    textures, sizes (down to a few pixels more than the border) and feature budgets:
    the keypoints (positions, angles, responses) and descriptors bit for bit."""
    from kcmc_amd import orb

    rng = np.random.default_rng(9000 + seed)
    F, H, W = int(rng.integers(1, 4)), int(rng.integers(36, 420)), int(rng.integers(36, 520))
    cell = int(rng.choice([2, 4, 8]))
    imgs = []
    for _ in range(F):
        lo = rng.integers(0, 256, (H // cell + 2, W // cell + 2)).astype(np.float64)
        img = np.kron(lo, np.ones((cell, cell)))[:H, :W] + rng.normal(0, float(rng.choice([0, 6, 20])), (H, W))
        imgs.append(np.clip(img, 0, 255).astype(np.uint8))
    imgs = np.stack(imgs)
    nf = int(rng.choice([1, 7, 100, 500, 2000]))
    k = stages.detect_orb(_t(imgs, dev), orb.OrbParams(n_features=nf))
    kp, des, cnt = k.kp.cpu().numpy(), k.des.cpu().numpy(), k.count.cpu().numpy()
    for f in range(F):
        rkp, rdes = oracle.orb_detect(imgs[f], n_features=nf, pattern=orb.rotated_patterns(), bin_cs=orb.bin_edges())
        assert cnt[f] == len(rkp), (seed, f, cnt[f], len(rkp))
        assert np.array_equal(kp[f, :cnt[f]], rkp), (seed, f)
        assert np.array_equal(des[f, :cnt[f]], rdes), (seed, f)


@pytest.mark.parametrize("seed", range(4))
def test_multidevice_split_fuzz(dev, seed):
    """VideoAligner over 2-5 slabs on cuda:0 (DEVICES = [0] * k) against one slab, with
    random frame counts (fewer frames than slabs included), model-less runs of frames at
    random places (gaps that cross slab boundaries), the model and the frame rate
    (temporal downsampling) drawn at random: identical arrays."""
    from kcmc_amd import VideoAligner, synthetic

    rng = np.random.default_rng(9500 + seed)
    model = str(rng.choice(["euclidean", "affine"]))
    rate = int(rng.choice([1, 2]))
    n_sample = int(rng.integers(2, 18))
    H, W = 72, 120
    ks = synthetic.make_keypoints(n_sample, 120, 32, (H, W), seed=9600 + seed, model=model)
    for f in rng.choice(n_sample, int(rng.integers(0, n_sample // 2 + 1)), replace=False):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ks.des_q[a:b] = rng.integers(0, 256, (1, 32), dtype=np.uint8)  # no ratio survivor: no model
    base = synthetic.make_texture((H, W), seed=seed)
    frames = np.ascontiguousarray(np.stack([np.roll(base, (f, 3 * f), axis=(0, 1))
                                            for f in range(n_sample * rate - rate // 2)]))
    kq = [ks.kp_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(n_sample)]
    dq = [ks.des_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(n_sample)]
    out = []
    for k in (1, int(rng.integers(2, 6))):
        class VA(VideoAligner):
            DEVICES = [0] * k
            RANSAC_MODEL = model
            N_KP_GLOBAL_MIN = 3

        va = VA()
        try:
            res = va.align_keypoints(frames, ks.kp_tpl, ks.des_tpl, kq, dq, n_kp_global=30, frame_rate=100 * rate)
        except VideoAligner.AlignmentError as e:  # every frame model-less: the same error either way
            res = ("AlignmentError", str(e))
        out.append((res, getattr(va, "interpolated_idxs", None)))
    (r1, i1), (r2, i2) = out
    if isinstance(r1[0], str):
        assert r1 == r2
        return
    np.testing.assert_array_equal(r2[0], r1[0])
    np.testing.assert_array_equal(r2[1], r1[1])
    assert r2[2] == r1[2] and i2 == i1


@pytest.mark.parametrize("shape,persp", [((1, 4320, 7680), False), ((1, 4320, 7680), True), ((1, 2160, 3840, 4), False),
                                         ((2, 4097, 257), True)])
def test_warp_large_frames_vs_oracle(dev, shape, persp):
    """8K one-channel, 4K RGBA and a 4097-row strip: tile grids far beyond the configs',
    every tile path, bit for bit."""
    rng = np.random.default_rng(sum(shape) + persp)
    imgs = _values(rng, shape)
    F, H, W = shape[:3]
    Ms = np.stack([(_perspective if persp else _affine)(rng, H, W) for _ in range(F)])
    if persp:
        Ms[:, 2, :2] = rng.normal(0, 1e-6, (F, 2))
    fn = stages.warp_perspective_u16 if persp else stages.warp_affine_u16
    ref = oracle.warp_perspective_u16 if persp else oracle.warp_affine_u16
    out = fn(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], ref(imgs[f], Ms[f])), (shape, persp, f)


@pytest.mark.parametrize("seed", range(4))
def test_overlapped_slabs_fuzz(dev, seed):
    """The pipelined schedule (OverlappedSlabs: streams, events, slot reuse, device maps and
    the re-warp of model-less frames) on random slab sequences -- slab sizes that change from
    slab to slab, model-less runs anywhere, the match beside the warp or ahead of it, the
    three models, temporal downsampling, float or byte descriptors -- equal to align_slab
    slab by slab."""
    from kcmc_amd import pipeline, synthetic

    rng = np.random.default_rng(9700 + seed)
    model = str(rng.choice(["euclidean", "affine", "projective"]))
    rate = int(rng.choice([1, 1, 2]))
    descriptor = str(rng.choice(["u8", "u8", "f32"]))
    beside = bool(rng.integers(0, 2)) and descriptor == "u8"
    H, W = int(rng.integers(64, 200)), int(rng.integers(64, 260))
    cfg = pipeline.AlignConfig(n_kp_global=int(rng.integers(12, 60)), ransac_model=model, frame_downsample_rate=rate)
    slabs = []
    for k in range(int(rng.integers(1, 5))):
        S = int(rng.integers(3, 14))
        D = 32 if descriptor == "u8" else 48
        ks = synthetic.make_keypoints(S, int(rng.integers(60, 220)), D, (H, W), seed=9800 + 10 * seed + k, model=model,
                                      descriptor=descriptor)
        for f in rng.choice(S, int(rng.integers(0, S // 2 + 1)), replace=False):
            a, b = ks.q_off[f], ks.q_off[f + 1]  # one descriptor row: no ratio survivor, no model
            ks.des_q[a:b] = ks.des_q[a] if descriptor == "f32" else rng.integers(0, 256, (1, D), dtype=np.uint8)
        frames = torch.from_numpy(np.ascontiguousarray(np.stack(
            [np.roll(synthetic.make_texture((H, W), seed=k), (f, 2 * f), axis=(0, 1)) for f in range(S * rate)]))).to(dev)
        slabs.append(pipeline.SlabInputs(frames, _t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev),
                                         _t(ks.kp_q, dev), _t(ks.q_off, dev), ks.q_off))
    ref = []
    for s in slabs:
        try:
            ref.append(pipeline.align_slab(s, cfg))
        except Exception as e:  # noqa: BLE001 - the same error must come out of the pipeline
            ref.append(e)
    if any(isinstance(r, Exception) for r in ref):
        with pytest.raises(type(next(r for r in ref if isinstance(r, Exception)))):
            ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=beside)
            [ov.submit(s) for s in slabs] + ov.flush()
            ov.synchronize()
        return
    ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=beside)
    got = [ov.submit(s) for s in slabs]
    got = got[1:] + ov.flush()
    ov.synchronize()
    for r, g in zip(ref, got):
        assert np.array_equal(r.affines, g.affines, equal_nan=True), seed
        assert r.skipped == g.skipped and r.interpolated == g.interpolated, seed
        assert torch.equal(r.aligned, g.aligned), seed
