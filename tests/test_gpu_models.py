"""Parity of the affine / projective RANSAC and warpPerspective kernels (the extension
behind BASELINE configs 3-5) with scikit-image 0.18.3 goldens and the CPU oracle.
Inlier sets / winning trials bit-exact; parameters within 1e-4 relative (north_star;
observed ~1e-10); warped pixels bit-exact to the oracle."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden
from kcmc_amd import stages, synthetic

pytestmark = pytest.mark.gpu
MODELS = ["affine", "projective"]


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _csr(lists):
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    return off


def _run(dev, model, tpls, qs, rate=1.0, trials=1000, n_skip=3):
    off = _csr(qs)
    r = stages.ransac_model(_t(np.concatenate(qs).reshape(-1, 2), dev), _t(np.concatenate(tpls).reshape(-1, 2), dev),
                            _t(off, dev), off, model=model, trials=trials, spatial_rate=rate, n_skip=n_skip)
    return (off, r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool), r.n_inliers.cpu().numpy(),
            r.best_trial.cpu().numpy())


@pytest.mark.parametrize("model", MODELS)
def test_ransac_model_vs_skimage_golden(dev, model):
    g = load_golden("ransac_models_golden.npz")
    off = g[f"{model}_offsets"]
    F = len(off) - 1
    tpls = [g[f"{model}_kp_template"][off[f]:off[f + 1]] for f in range(F)]
    qs = [g[f"{model}_kp_query"][off[f]:off[f + 1]] for f in range(F)]
    o2, params, inl, nin, _ = _run(dev, model, tpls, qs)
    for f in range(F):
        ref = g[f"{model}_params"][f]
        if np.isnan(ref).any():
            assert np.isnan(params[f]).all(), f
            continue
        np.testing.assert_allclose(params[f], ref, rtol=1e-4, atol=1e-6, err_msg=str(f))
        np.testing.assert_allclose(params[f], ref, rtol=1e-6, atol=1e-8, err_msg=str(f))
        assert np.array_equal(inl[o2[f]:o2[f + 1]], g[f"{model}_inliers"][off[f]:off[f + 1]]), f
        assert nin[f] == g[f"{model}_n_inliers"][f], f


def _frames(rng, model, Ns):
    tpls, qs = [], []
    for N in Ns:
        tpl = rng.uniform(0, 1000, (N, 2))
        Hm = np.eye(3)
        Hm[:2, :2] += rng.normal(0, 0.01, (2, 2))
        Hm[:2, 2] = rng.normal(0, 5, 2)
        if model == "projective":
            Hm[2, :2] = rng.normal(0, 1e-5, 2)
        q = oracle._apply_h(np.linalg.inv(Hm), tpl) + rng.normal(0, rng.uniform(0.1, 1.5), (N, 2))
        out = rng.random(N) < rng.uniform(0, 0.6)
        q[out] = rng.uniform(0, 1000, (int(out.sum()), 2))
        tpls.append(tpl.astype(np.float32).astype(np.float64))
        qs.append(q.astype(np.float32).astype(np.float64))
    return tpls, qs


@pytest.mark.parametrize("model", MODELS)
def test_ransac_model_bit_exact_selection_vs_oracle(dev, model):
    """Same hypotheses and arithmetic as the C oracle -> identical winning trial and
    inlier set, including N > 128 (numpy's recursive pairwise order)."""
    rng = np.random.default_rng(71 if model == "affine" else 72)
    Ns = [5, 6, 8, 9, 20, 50, 100, 127, 128, 129, 136, 200, 256, 257, 300, 500, 1024]
    tpls, qs = _frames(rng, model, Ns)
    off, params, inl, nin, best = _run(dev, model, tpls, qs)
    for f in range(len(qs)):
        p, i_ref, bt, ni = oracle.ransac_model(qs[f], tpls[f], model)
        assert best[f] == bt, f
        assert nin[f] == ni, f
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), f
        np.testing.assert_allclose(params[f], p, rtol=1e-8, atol=1e-9, err_msg=str(f))


@pytest.mark.parametrize("model", MODELS)
@pytest.mark.parametrize("thresh", [2.0, 1e-120, 5e-5])
def test_ransac_model_two_phase_ties_and_exact_fallback(dev, model, thresh):
    """The two-phase scoring (counts through q < tq and fp32 S estimates, then numpy's
    pairwise S for the trials that can tie) against the oracle: nearly noise-free inlier
    sets (S near-ties), duplicated points (exact ties), N > 128, and the frames that fall
    back to exact scoring (threshold 1e-120: tq out of range; 5e-5: no inliers on noisy
    frames; exact integer data: S == 0)."""
    rng = np.random.default_rng(81 if model == "affine" else 82)
    tpls, qs = [], []
    for N, noise in [(40, 1e-9), (90, 1e-6), (90, 0.3), (150, 1e-7), (12, 0.0)]:
        tpl = rng.uniform(0, 1000, (N, 2))
        Hm = np.eye(3)
        Hm[:2, :2] += rng.normal(0, 0.01, (2, 2))
        Hm[:2, 2] = rng.normal(0, 5, 2)
        if model == "projective":
            Hm[2, :2] = rng.normal(0, 1e-5, 2)
        if noise:
            q = oracle._apply_h(np.linalg.inv(Hm), tpl) + rng.normal(0, noise, (N, 2))
        else:
            tpl = np.round(tpl)
            q = tpl - np.array([3.0, 1.0])
        if N == 90 and noise == 0.3:
            q[45:], tpl[45:] = q[:45], tpl[:45]
        tpls.append(tpl)
        qs.append(q)
    off = _csr(qs)
    r = stages.ransac_model(_t(np.concatenate(qs), dev), _t(np.concatenate(tpls), dev), _t(off, dev), off,
                            model=model, residual_threshold=thresh, n_skip=3)
    params, inl = r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool)
    nin, best = r.n_inliers.cpu().numpy(), r.best_trial.cpu().numpy()
    for f in range(len(qs)):
        p, i_ref, bt, ni = oracle.ransac_model(qs[f], tpls[f], model, thresh=thresh)
        assert best[f] == bt, f
        assert nin[f] == ni, f
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), f
        if model == "projective" and ni < 4:
            # skimage's refit on < 4 inliers is underdetermined (a 3-D null space of the
            # 2N x 9 system): its params are whatever LAPACK's SVD returns, unpinned
            continue
        np.testing.assert_allclose(params[f], p, rtol=1e-8, atol=1e-9, equal_nan=True, err_msg=str(f))


@pytest.mark.parametrize("model", MODELS)
def test_ransac_model_skips_degenerate_and_scales(dev, model):
    rng = np.random.default_rng(73)
    tpl = rng.uniform(0, 100, (12, 2))
    same = np.repeat(tpl[:1], 12, 0)
    ms = 3 if model == "affine" else 4
    tpls = [tpl, tpl[:2], tpl[:0], tpl]
    qs = [same, tpl[:2] + 1, tpl[:0], tpl - 3.0]
    off, params, inl, nin, best = _run(dev, model, tpls, qs, rate=2.0)
    assert np.isnan(params[0]).all() and nin[0] == 0 and best[0] == -1
    assert np.isnan(params[1]).all() and np.isnan(params[2]).all()  # N < N_KP_FRAME_SKIP
    expect = np.array([[1, 0, 6.0], [0, 1, 6.0], [0, 0, 1]])  # translation 3 * spatial rate 2
    np.testing.assert_allclose(params[3], expect, atol=1e-8)
    with pytest.raises(ValueError):  # skimage: min_samples must be < number of samples
        _run(dev, model, [tpl[:ms]], [tpl[:ms] + 1])


@pytest.mark.parametrize("model", MODELS)
def test_ransac_model_gather_mode_matches_contiguous(dev, model):
    rng = np.random.default_rng(74)
    n_tpl, F = 80, 6
    n_skip = 5 if model == "projective" else 4
    kp_tpl = rng.uniform(0, 500, (n_tpl, 2))
    kp_ord = kp_tpl[None] * 1.01 + rng.normal(0, 0.5, (F, n_tpl, 2)) + 2.0
    lists = [rng.permutation(n_tpl)[: int(rng.integers(0, 60))].astype(np.int32) for _ in range(F)]
    off = _csr(lists)
    r = stages.ransac_model(_t(kp_ord.reshape(-1, 2), dev), _t(kp_tpl, dev), _t(off, dev), off, model=model,
                            pt_idx=_t(np.concatenate(lists), dev), src_frame_stride=n_tpl, n_skip=n_skip)
    _, p2, _, _, _ = _run(dev, model, [kp_tpl[L] for L in lists], [kp_ord[f][L] for f, L in enumerate(lists)],
                          n_skip=n_skip)
    np.testing.assert_array_equal(r.params.cpu().numpy(), p2)


# ------------------------------------------------------------------ warpPerspective
def _homographies(rng, F, H, W):
    Ms = []
    for _ in range(F):
        Hm = np.eye(3)
        Hm[:2, :2] += rng.normal(0, 0.02, (2, 2))
        Hm[:2, 2] = rng.normal(0, 6, 2)
        Hm[2, :2] = rng.normal(0, 1e-2 / max(H, W), 2)
        Ms.append(Hm)
    return np.stack(Ms)


@pytest.mark.parametrize("shape", [(1, 5, 7), (3, 64, 128), (2, 67, 131), (2, 130, 257), (1, 1080, 1920)])
def test_warp_perspective_matches_oracle(dev, shape):
    F, H, W = shape
    rng = np.random.default_rng(H * W + 1)
    imgs = rng.integers(0, 65536, shape).astype(np.uint16)
    Ms = _homographies(rng, F, H, W)
    out = stages.warp_perspective_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_perspective_u16(imgs[f], Ms[f])), f


def test_warp_perspective_extreme_maps_and_inverse(dev):
    """Horizon inside the frame (denominator changes sign -> direct gather), singular
    map, strong zoom, frames far outside, and WARP_INVERSE_MAP."""
    rng = np.random.default_rng(81)
    H, W = 200, 300
    img = rng.integers(0, 65536, (H, W)).astype(np.uint16)
    Ms = [np.eye(3), np.array([[1, 0.1, 5], [0.02, 1, -3], [0.004, 0.001, 1.0]]),
          np.zeros((3, 3)), np.array([[2.5, 0, -100], [0, 2.5, -80], [0, 0, 1.0]]),
          np.array([[1, 0, 5000], [0, 1, 0], [0, 0, 1.0]]),
          np.array([[0.9, 0.05, 3], [-0.04, 1.1, 2], [-2e-4, 1e-4, 1]])]
    imgs = np.broadcast_to(img, (len(Ms), H, W)).copy()
    for inv in (False, True):
        out = stages.warp_perspective_u16(_t(imgs, dev), _t(np.stack(Ms), dev), inverse_map=inv).cpu().numpy()
        for f, M in enumerate(Ms):
            assert np.array_equal(out[f], oracle.warp_perspective_u16(img, M, inverse_map=inv)), (f, inv)
    assert np.array_equal(out[0], img)


@pytest.mark.parametrize("C", [3, 4])
def test_warp_perspective_multichannel(dev, C):
    rng = np.random.default_rng(90 + C)
    imgs = rng.integers(0, 65536, (2, 60, 90, C)).astype(np.uint16)
    Ms = _homographies(rng, 2, 60, 90)
    out = stages.warp_perspective_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(2):
        assert np.array_equal(out[f], oracle.warp_perspective_u16(imgs[f], Ms[f]))


def test_warp_perspective_of_affine_close_to_affine_path(dev):
    """An affine homography through warpPerspective differs from warpAffine only by the
    coordinate rounding (double per pixel vs 1/1024 fixed point): at most a 1/32-px tap
    shift, i.e. a few LSB on a smooth ramp."""
    H, W = 120, 160
    yy, xx = np.mgrid[0:H, 0:W]
    img = (20000 + 50 * xx + 30 * yy).astype(np.uint16)
    A = synthetic.rigid(0.01, 3.3, -2.1)
    Hm = np.vstack([A, [0, 0, 1]])
    a = stages.warp_affine_u16(_t(img[None], dev), _t(A[None], dev)).cpu().numpy()[0].astype(int)
    p = stages.warp_perspective_u16(_t(img[None], dev), _t(Hm[None], dev)).cpu().numpy()[0].astype(int)
    inner = (slice(8, H - 8), slice(8, W - 8))
    assert np.abs(a[inner] - p[inner]).max() <= 8


# ------------------------------------------------------------------ whole slab
@pytest.mark.parametrize("model", MODELS)
def test_slab_end_to_end_with_model(dev, model):
    """match -> consensus -> affine/projective RANSAC -> gap filling -> warp, checked
    frame by frame against the oracle (RANSAC on the same consensus point lists, warp of
    the resulting maps)."""
    from kcmc_amd import pipeline

    F, H, W = 12, 256, 320
    ks = synthetic.make_keypoints(F, 300, 61, (H, W), seed=11, model=model)
    base = synthetic.make_texture((H, W), seed=12)
    frames = torch.from_numpy(np.broadcast_to(base, (F, H, W)).copy()).to(dev)
    inp = pipeline.SlabInputs(frames, _t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev),
                              _t(ks.q_off, dev), ks.q_off)
    cfg = pipeline.AlignConfig(n_kp_global=60, ransac_model=model)
    res = pipeline.align_slab(inp, cfg, keep_intermediates=True)
    torch.cuda.synchronize()
    kq = res.match.kp_ordered.cpu().numpy()
    po, pi = res.consensus.pt_off, res.consensus.pt_idx
    out = res.aligned.cpu().numpy()
    assert res.affines.shape[1:] == ((2, 3) if model == "affine" else (3, 3))
    n_fit = 0
    for f in range(F):
        L = pi[po[f]:po[f + 1]]
        p, _, _, _ = oracle.ransac_model(kq[f][L], ks.kp_tpl[L], model)
        if model == "affine":
            p = p[:2]
        if not np.isnan(p).any():
            n_fit += 1
            np.testing.assert_allclose(res.affines[f], p, rtol=1e-6, atol=1e-8, err_msg=str(f))
            # the recovered map is the ground truth up to the keypoint noise
            assert np.abs(res.affines[f][:2, 2] - ks.gt[f][:2, 2]).max() < 1.0
        ref = (oracle.warp_affine_u16(base, res.affines[f]) if model == "affine"
               else oracle.warp_perspective_u16(base, res.affines[f]))
        assert np.array_equal(out[f], ref), f
    assert n_fit == F


def test_video_aligner_model_selector(dev):
    from kcmc_amd import VideoAligner

    class AffineAligner(VideoAligner):
        RANSAC_MODEL = "affine"

    F, H, W = 6, 128, 160
    ks = synthetic.make_keypoints(F, 200, 32, (H, W), seed=13, model="affine")
    imgs = np.broadcast_to(synthetic.make_texture((H, W), seed=14), (F, H, W)).copy()
    kps = [ks.kp_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(F)]
    des = [ks.des_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(F)]
    aligned, eu, skipped = AffineAligner().align_keypoints(imgs, ks.kp_tpl, ks.des_tpl, kps, des, n_kp_global=50)
    assert aligned.shape == imgs.shape and eu.shape == (F, 3) and skipped == []
    np.testing.assert_allclose(eu[:, :2], ks.gt[:, :, 2], atol=1.0)


# ------------------------------------------------------------ float descriptors (K1f)
@pytest.mark.parametrize("D", [1, 3, 64, 100, 128])
def test_knn2_f32_matches_oracle(dev, D):
    """MFMA candidate search + exact re-ranking == exact brute force (indices and
    distances bit-exact), including exact duplicates (ties -> lower index) and runs of
    4+ equidistant rows, which take the exact fallback path."""
    rng = np.random.default_rng(100 + D)
    n_tpl = 300
    tpl = rng.normal(0, 1, (n_tpl, D)).astype(np.float32)
    frames = []
    for f, n_q in enumerate([700, 1500, 3, 2, 1, 0, 64, 65, 200]):
        q = rng.normal(0, 1, (n_q, D)).astype(np.float32)
        if n_q > 40:
            q[: n_q // 3] = tpl[rng.integers(0, n_tpl, n_q // 3)] + rng.normal(0, 0.05, (n_q // 3, D)).astype(np.float32)
            q[10] = q[11] = q[12] = q[13] = q[14] = tpl[5]  # five exact copies of one template row
            q[20] = q[3]
        frames.append(q)
    off = _csr(frames)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames).reshape(-1, D), dev), _t(off, dev),
                                 int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_l2f32(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


@pytest.mark.parametrize("scale", [1e-3, 37.0, 1e4])
def test_knn2_f32_scaled_and_near_ties(dev, scale):
    """The bf16x3 candidate search's error bound scales with the descriptor norms: scaled
    descriptors, frame rows that differ from a template row by one bf16 ulp of a single
    element (near-ties below the split's resolution) and rows of mixed magnitude."""
    rng = np.random.default_rng(int(scale * 10))
    n_tpl, D = 200, 128
    tpl = (rng.normal(0, 1, (n_tpl, D)) * scale).astype(np.float32)
    frames = []
    for n_q in [900, 130, 33]:
        q = (rng.normal(0, 1, (n_q, D)) * scale).astype(np.float32)
        q[: n_q // 4] = tpl[rng.integers(0, n_tpl, n_q // 4)]
        for k in range(n_q // 4, n_q // 4 + 12):  # copies of template row 7 nudged in one element
            q[k] = tpl[7]
            q[k, k % D] = np.nextafter(q[k, k % D], np.float32(np.inf), dtype=np.float32)
        q[-3:] *= np.float32(1e-2)  # small-norm rows
        frames.append(q)
    off = _csr(frames)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames).reshape(-1, D), dev), _t(off, dev),
                                 int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_l2f32(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


def test_match_frames_f32_vs_oracle(dev):
    """SIFT-style float descriptors through knn + the reference's filters (VA:196-214)."""
    ks = synthetic.make_keypoints(12, 400, 128, (1080, 1920), seed=15, descriptor="f32")
    m = stages.match_frames(_t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev),
                            _t(ks.q_off, dev), ks.q_off)
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kqo = m.kp_ordered.cpu().numpy()
    cnt = m.counts.cpu().numpy()
    for f in range(12):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        idx, dist = oracle.knn2_l2f32(ks.des_tpl, ks.des_q[a:b])
        s, kq, c = oracle.filter_matches(idx, dist, ks.kp_tpl, ks.kp_q[a:b])
        kept = [i for i in range(400) if (bits[f, i >> 5] >> (i & 31)) & 1]
        assert kept == sorted(s)
        assert np.array_equal(kqo[f], kq)
        assert cnt[f].tolist() == list(c)
        assert len(kept) > 250


@pytest.mark.parametrize("n_q", [2, 3, 70])
def test_knn2_f32_frame_beyond_fp16_range_goes_to_fallback(dev, n_q):
    """A frame whose values are ~5e4 x the template's largest element overflows the fp16
    tile image (flagged): every template row must come from the exact fallback, also when
    the overflowed values would otherwise read as 'fewer than two frame rows' (round 5: the
    fuzz sweep found such frames returned -1 / FLT_MAX)."""
    rng = np.random.default_rng(n_q)
    tpl = rng.normal(0, 1e-3, (300, 113)).astype(np.float32)
    frames = [rng.normal(0, 1e-3, (40, 113)).astype(np.float32), rng.normal(0, 50.0, (n_q, 113)).astype(np.float32),
              rng.normal(0, 1e-3, (9, 113)).astype(np.float32)]
    off = np.zeros(4, np.int32)
    off[1:] = np.cumsum([len(q) for q in frames])
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames), dev), _t(off, dev), int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_l2f32(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


@pytest.mark.parametrize("kind", ["u8", "hamming", "f32", "u8_big"])
def test_knn_then_filter_on_two_streams_equals_match_frames(dev, kind):
    """knn_frames on one stream + filter_matches on another ordered after it (the c5
    schedule: knn on the kernel stream, filter + vote on the analysis stream) =
    match_frames, bit for bit: L2 u8, Hamming, float32 and n_tpl 4096 (the filter's
    workgroup kernel)."""
    if kind == "f32":
        ks = synthetic.make_keypoints(9, 300, 128, (270, 480), seed=16, descriptor="f32")
    elif kind == "u8_big":
        ks = synthetic.make_keypoints(3, 4096, 61, (512, 512), seed=17)
    else:
        ks = synthetic.make_keypoints(9, 500, 32, (1080, 1920), seed=18)
    norm = "hamming" if kind == "hamming" else "l2"
    args = (_t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev), _t(ks.q_off, dev), ks.q_off)
    ref = stages.match_frames(*args, norm=norm)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s1.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s1):
        knn = stages.knn_frames(*args, norm=norm, stream=s1.cuda_stream)
    s2.wait_stream(s1)
    with torch.cuda.stream(s2):
        got = stages.filter_matches(knn, args[1], args[3], args[4], stream=s2.cuda_stream)
    torch.cuda.current_stream(dev).wait_stream(s2)
    for name in ("idx", "dist", "kp_ordered", "keep_bits", "counts"):
        assert torch.equal(getattr(ref, name), getattr(got, name)), name
    with pytest.raises(ValueError, match="shapes disagree"):
        stages.filter_matches((knn[0][:1], knn[1]), args[1], args[3], args[4])


# ------------------------------------------------------------ f2: normalisation
def test_brightest_px_and_max_scale_vs_reference_golden(dev):
    g = load_golden("preprocess_golden.npz")
    for k in range(int(g["n_cases"])):
        imgs = g[f"p{k}_images"]
        b = stages.brightest_px(_t(imgs, dev))
        assert b == g[f"p{k}_brightest"], k
        u8 = stages.max_scale_u8(_t(imgs, dev), b).cpu().numpy()
        assert np.array_equal(u8, g[f"p{k}_u8"]), k


@pytest.mark.parametrize("shape,hi", [((3, 37, 41), 65536), ((50, 128, 128), 4096), ((2, 1080, 1920), 65536),
                                      ((5, 7, 3), 2), ((1, 1, 1), 65536)])
def test_brightest_px_matches_numpy(dev, shape, hi):
    rng = np.random.default_rng(int(np.prod(shape)) + hi)
    imgs = rng.integers(0, hi, shape).astype(np.uint16)
    if imgs.size > 100:
        imgs.reshape(-1)[rng.integers(0, imgs.size, 20)] = 65000  # hot pixels above the 99.99th percentile
    t = _t(imgs, dev)
    for q in (99.99, 50.0, 0.0, 100.0):
        assert stages.brightest_px(t, q) == np.percentile(imgs, q), q
    b = np.percentile(imgs, 99.99)
    ref = np.clip(imgs / b * 255, a_min=0, a_max=255).astype(np.uint8)
    assert np.array_equal(stages.max_scale_u8(t, b).cpu().numpy(), ref)


def test_brightest_px_concentrated_values(dev):
    # the bench texture: most values in a few coarse bins (the histogram's worst case for
    # atomic collisions), plus a stack where every value is identical
    imgs = np.stack([synthetic.make_texture((360, 480), seed=s) for s in range(4)])
    t = _t(imgs, dev)
    for q in (99.99, 50.0, 1.0):
        assert stages.brightest_px(t, q) == np.percentile(imgs, q), q
    same = np.full((3, 64, 64), 2047, np.uint16)
    assert stages.brightest_px(_t(same, dev), 99.99) == 2047.0


# ------------------------------------------------------------ f1: detection
def _texture_u8(rng, H, W, cell=4, noise=12):
    lo = rng.integers(0, 256, (H // cell + 2, W // cell + 2)).astype(np.float64)
    img = np.kron(lo, np.ones((cell, cell)))[:H, :W] + rng.normal(0, noise, (H, W))
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape,nf", [((3, 120, 200), 500), ((2, 256, 320), 40), ((1, 1080, 1920), 500)])
def test_orb_detect_matches_oracle(dev, shape, nf):
    from kcmc_amd import orb

    rng = np.random.default_rng(shape[1] + nf)
    F, H, W = shape
    imgs = np.stack([_texture_u8(rng, H, W) for _ in range(F)])
    if F >= 2:
        imgs[1, :, : W // 2] = 100  # a flat half: no corners there
    if F == 3:
        imgs[2] = np.tile(_texture_u8(rng, 40, 40), (3, 5))[:H, :W]  # repeated tiles: equal Harris -> ties
    k = stages.detect_orb(_t(imgs, dev), orb.OrbParams(n_features=nf))
    kp, des, cnt = k.kp.cpu().numpy(), k.des.cpu().numpy(), k.count.cpu().numpy()
    for f in range(F):
        rkp, rdes = oracle.orb_detect(imgs[f], n_features=nf, pattern=orb.rotated_patterns(), bin_cs=orb.bin_edges())
        assert cnt[f] == len(rkp), (f, cnt[f], len(rkp))
        assert np.array_equal(kp[f, :cnt[f]], rkp), f
        assert np.array_equal(des[f, :cnt[f]], rdes), f
        assert cnt[f] > 0
    flat = stages.detect_orb(_t(np.full((1, 64, 64), 7, np.uint8), dev))
    assert flat.count.cpu().numpy()[0] == 0


def test_orb_keypoints_feed_the_matcher(dev):
    """Detect on a frame and on its shifted copy, match through the reference's
    matcher + filters, and recover the shift with RANSAC: the GPU front end end to end."""
    from kcmc_amd import orb, pipeline

    rng = np.random.default_rng(5)
    H, W = 240, 320
    base = _texture_u8(rng, H + 20, W + 20)
    tpl = base[10:10 + H, 10:10 + W]
    frames = np.stack([base[10 + dy:10 + dy + H, 10 + dx:10 + dx + W] for dy, dx in ((0, 0), (3, -2), (-4, 5))])
    kt = stages.detect_orb(_t(tpl, dev))
    kq = stages.detect_orb(_t(frames, dev))
    n_t = int(kt.count.cpu()[0])
    kp_q, des_q, q_off, q_off_host = stages.keypoints_csr(kq)
    inp = pipeline.SlabInputs(_t(frames.astype(np.uint16), dev), kt.des[0, :n_t].contiguous(),
                              kt.kp[0, :n_t].contiguous(), des_q, kp_q, q_off, q_off_host)
    res = pipeline.align_slab(inp, pipeline.AlignConfig(n_kp_global=60), keep_intermediates=True)
    # frame content at (x, y) is the template at (x + dx, y + dy): frame->template map translates by (dx, dy)
    for f, (dy, dx) in enumerate(((0, 0), (3, -2), (-4, 5))):
        np.testing.assert_allclose(res.affines[f][:, 2], [dx, dy], atol=1e-6)
