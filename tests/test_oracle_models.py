"""Pin the oracle of the affine / projective extension (BASELINE configs 3-5):
against scikit-image 0.18.3 itself (tests/golden/make_golden_models.py), against the
operation-for-operation SVD restatement, and -- for warpPerspective, whose OpenCV
oracle is absent from this image -- against an independent pure-Python restatement."""
import numpy as np
import pytest

import oracle
from conftest import load_golden


@pytest.mark.parametrize("model", ["affine", "projective"])
def test_ransac_model_oracle_vs_skimage_golden(model):
    """The closed-form hypothesis loop + numpy SVD refit reproduce skimage 0.18.3 on
    every golden frame (inlier sets bit-exact, params within 1e-6 relative)."""
    g = load_golden("ransac_models_golden.npz")
    off = g[f"{model}_offsets"]
    for f in range(len(off) - 1):
        a, b = off[f], off[f + 1]
        p, inl, bt, ni = oracle.ransac_model(g[f"{model}_kp_query"][a:b], g[f"{model}_kp_template"][a:b], model)
        ref = g[f"{model}_params"][f]
        if np.isnan(ref).any():
            assert np.isnan(p).all(), f
            continue
        assert np.array_equal(inl, g[f"{model}_inliers"][a:b]), f
        assert ni == g[f"{model}_n_inliers"][f]
        np.testing.assert_allclose(p, ref, rtol=1e-6, atol=1e-9, err_msg=str(f))


@pytest.mark.parametrize("model", ["affine", "projective"])
def test_ransac_model_closed_form_agrees_with_svd_restatement(model):
    rng = np.random.default_rng(5 if model == "affine" else 6)
    for N in (5, 9, 40, 150):
        tpl = rng.uniform(0, 400, (N, 2))
        Hm = np.array([[1.01, 0.02, 3], [-0.01, 0.99, -2], [2e-5 if model == "projective" else 0, 0, 1]])
        q = oracle._apply_h(np.linalg.inv(Hm), tpl) + rng.normal(0, 0.4, (N, 2))
        q[: N // 4] = rng.uniform(0, 400, (N // 4, 2))
        p, inl, _, _ = oracle.ransac_model(q, tpl, model)
        p2, inl2 = oracle.ransac_model_skimage(q, tpl, model)
        assert np.array_equal(inl, inl2)
        np.testing.assert_allclose(p, p2, rtol=1e-9, atol=1e-9)


def test_hypothesis_stream_three_and_four_samples():
    """skimage draws choice(N, k, replace=False) == permutation(N)[:k] per trial."""
    for k in (3, 4):
        for n in (5, 17, 300):
            rs = np.random.RandomState(42)
            ref = np.array([rs.permutation(n)[:k] for _ in range(50)])
            assert np.array_equal(oracle.hypothesis_table(n, 50, 42, k), ref)


def test_perspective_inverse_matches_numpy():
    rng = np.random.default_rng(7)
    for _ in range(20):
        M = np.eye(3) + rng.normal(0, 0.1, (3, 3))
        np.testing.assert_allclose(oracle.invert_perspective(M), np.linalg.inv(M), rtol=1e-10, atol=1e-12)
    assert not oracle.invert_perspective(np.zeros((3, 3))).any()


def _warp_perspective_py(img, M):
    """Independent pure-Python restatement of the classic warpPerspective path
    (WarpPerspectiveInvoker + remapBilinear), small images only."""
    Mi = oracle.invert_perspective(M)
    H, W = img.shape
    bh0 = min(16, H)
    bw0 = min(1024 // bh0, W)
    out = np.zeros_like(img)
    tab = [(np.float32(1) - np.float32(i) * np.float32(1 / 32), np.float32(i) * np.float32(1 / 32)) for i in range(32)]
    for y in range(H):
        for x in range(W):
            xo = (x // bw0) * bw0
            x1 = x - xo
            X0 = Mi[0, 0] * xo + Mi[0, 1] * y + Mi[0, 2]
            Y0 = Mi[1, 0] * xo + Mi[1, 1] * y + Mi[1, 2]
            W0 = Mi[2, 0] * xo + Mi[2, 1] * y + Mi[2, 2]
            w = W0 + Mi[2, 0] * x1
            w = 32 / w if w else 0.0
            X = int(np.rint((X0 + Mi[0, 0] * x1) * w))
            Y = int(np.rint((Y0 + Mi[1, 0] * x1) * w))
            sx, sy, fx, fy = X >> 5, Y >> 5, X & 31, Y & 31
            v = [np.float32(img[yy, xx]) if 0 <= xx < W and 0 <= yy < H else np.float32(0)
                 for yy, xx in ((sy, sx), (sy, sx + 1), (sy + 1, sx), (sy + 1, sx + 1))]
            wts = [tab[fy][0] * tab[fx][0], tab[fy][0] * tab[fx][1], tab[fy][1] * tab[fx][0], tab[fy][1] * tab[fx][1]]
            acc = np.float32(0)
            for vv, ww in zip(v, wts):
                acc = np.float32(acc + np.float32(vv * ww))
            out[y, x] = min(max(int(np.rint(acc)), 0), 65535)
    return out


def test_warp_perspective_matches_independent_python_restatement():
    rng = np.random.default_rng(8)
    img = rng.integers(0, 65536, (23, 70)).astype(np.uint16)  # W > 64: two column blocks
    for M in (np.array([[1.0, 0.05, 2.3], [-0.03, 0.97, 1.1], [1e-3, -5e-4, 1.0]]), np.eye(3)):
        assert np.array_equal(oracle.warp_perspective_u16(img, M), _warp_perspective_py(img, M))


def test_warp_perspective_identity_and_affine_homography_known_answers():
    rng = np.random.default_rng(9)
    img = rng.integers(0, 65536, (17, 19)).astype(np.uint16)
    assert np.array_equal(oracle.warp_perspective_u16(img, np.eye(3)), img)
    # integer translation: dst(x, y) = src(x - 2, y - 1), zeros where that leaves the image
    T = np.array([[1.0, 0, 2], [0, 1, 1], [0, 0, 1]])
    out = oracle.warp_perspective_u16(img, T)
    assert np.array_equal(out[1:, 2:], img[:-1, :-2])
    assert not out[0].any() and not out[:, :2].any()


# ------------------------------------------------------------ float descriptors
def test_knn2_l2f32_oracle_matches_numpy_definition():
    rng = np.random.default_rng(10)
    q = rng.normal(0, 1, (40, 128)).astype(np.float32)
    t = rng.normal(0, 1, (300, 128)).astype(np.float32)
    t[7] = t[3]  # exact duplicates -> equal distances, lower index first
    q[5] = t[3]
    idx, dist = oracle.knn2_l2f32(q, t)
    d = np.sqrt(((q[:, None, :].astype(np.float64) - t[None].astype(np.float64)) ** 2).sum(-1).astype(np.float32))
    for i in range(len(q)):
        order = sorted(range(len(t)), key=lambda j: (d[i, j], j))[:2]
        assert idx[i].tolist() == order
        np.testing.assert_allclose(dist[i], d[i, order], rtol=1e-6)
    assert idx[5].tolist() == [3, 7] and dist[5, 0] == 0.0 and dist[5, 1] == 0.0


def test_knn2_l2f32_oracle_degenerate_train_sets():
    q = np.ones((3, 16), np.float32)
    idx, dist = oracle.knn2_l2f32(q, np.zeros((1, 16), np.float32))
    assert idx[:, 1].tolist() == [-1] * 3 and (dist[:, 1] == np.finfo(np.float32).max).all()
    idx, _ = oracle.knn2_l2f32(q, np.zeros((0, 16), np.float32))
    assert (idx == -1).all()
