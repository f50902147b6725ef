"""End-to-end parity of the batched hot path and of the reference-shaped API."""
import logging

import numpy as np
import pytest
import torch

import oracle
from conftest import distinct_frames, load_golden
from kcmc_amd import VideoAligner, pipeline, stages, synthetic

pytestmark = pytest.mark.gpu


def _split(flat, off):
    return [flat[off[i]:off[i + 1]] for i in range(len(off) - 1)]


class _KP:
    def __init__(self, x, y):
        self.pt = (float(x), float(y))


class _RegistryDetector:
    """Test stand-in for cv2.AKAZE: returns the golden keypoints registered for an image."""

    registry = {}

    def detectAndCompute(self, image, mask):
        kp, des = self.registry[np.ascontiguousarray(image).tobytes()]
        return [_KP(x, y) for x, y in kp], des


def test_align_keypoints_vs_reference_pipeline_golden():
    g = load_golden("pipeline_golden.npz")
    qo = g["q_offsets"]
    va = VideoAligner()
    aligned, eu, skipped = va.align_keypoints(g["images"], g["kp_template"], g["des_template"],
                                              _split(g["kp_query"], qo), _split(g["des_query"], qo),
                                              int(g["n_kp_global"]), frame_rate=30)
    assert skipped == g["skipped"].tolist()
    assert va.interpolated_idxs == g["interpolated"].tolist()
    np.testing.assert_allclose(eu, g["euclidean"], rtol=1e-4, atol=1e-6)
    assert np.array_equal(aligned, g["aligned"])


def test_align_images_with_registered_detector_vs_golden(monkeypatch):
    g = load_golden("pipeline_golden.npz")
    imgs = g["images"]
    F = len(imgs)
    b = VideoAligner._get_brightest_px(imgs)
    t_idx = int(F * VideoAligner.TEMPLATE_FRAME_LOC)
    i8, t8 = VideoAligner._max_scale_images(imgs, imgs[t_idx], b, np.uint8)
    qo = g["q_offsets"]
    kq, dq = _split(g["kp_query"], qo), _split(g["des_query"], qo)
    reg = {t8.tobytes(): (g["kp_template"], g["des_template"])}
    for f in range(F):
        reg[np.ascontiguousarray(i8[f]).tobytes()] = (kq[f], dq[f])
    _RegistryDetector.registry = reg
    monkeypatch.setitem(VideoAligner.DETECTOR_CONSTRUCTOR_DICT, "akaze", _RegistryDetector)
    aligned, eu, skipped = VideoAligner().align_images(imgs, n_kp_global=int(g["n_kp_global"]),
                                                       detector_algorithm="akaze", frame_rate=30)
    assert skipped == g["skipped"].tolist()
    np.testing.assert_allclose(eu, g["euclidean"], rtol=1e-4, atol=1e-6)
    assert np.array_equal(aligned, g["aligned"])
    # patch crop semantics (VA:153-157): axis 1 by x, axis 2 by y
    a2, _, _ = VideoAligner().align_images(imgs, int(g["n_kp_global"]), "akaze", 30, patch=(3, 5, 10, 20))
    assert np.array_equal(a2, g["aligned"][:, 3:13, 5:25])


def test_per_frame_helpers_match_reference_golden(monkeypatch):
    g = load_golden("ransac_golden.npz")
    off = g["offsets"]
    for f in range(0, len(off) - 1, 5):
        tpl, q = g["kp_template"][off[f]:off[f + 1]], g["kp_query"][off[f]:off[f + 1]]
        a = VideoAligner._compute_euclidean_affine(tpl, q, int(g["spatial_rate"][f]))
        ref = g["affine"][f]
        if np.isnan(ref).any():
            assert np.isnan(a).all()
        else:
            np.testing.assert_allclose(a, ref, rtol=1e-4, atol=1e-6)
    m = load_golden("match_golden_akaze.npz")
    qo, so = m["q_offsets"], m["kp_idxs_offsets"]
    reg = {}
    for f in range(4):
        img = np.full((4, 4), f, np.uint8)
        reg[img.tobytes()] = (m["kp_query"][qo[f]:qo[f + 1]], m["des_query"][qo[f]:qo[f + 1]])
    _RegistryDetector.registry = reg
    monkeypatch.setitem(VideoAligner.DETECTOR_CONSTRUCTOR_DICT, "akaze", _RegistryDetector)
    for f in range(4):
        s, kq, log = VideoAligner._get_frame_keypoints(f, np.full((4, 4), f, np.uint8), m["kp_template"],
                                                       m["des_template"], "akaze")
        assert list(s) == m["kp_idxs_setorder"][so[f]:so[f + 1]].tolist()
        assert np.array_equal(kq, m["kp_query_ordered"][f])
        assert [int(l.split()[0]) for l in log.split("\n")[1:]] == m["log_counts"][f].tolist()
    img = np.random.default_rng(0).integers(0, 65536, (40, 50)).astype(np.uint16)
    M = synthetic.rigid(0.05, 2.5, -1.25)
    assert np.array_equal(VideoAligner._apply_affine(img, M), oracle.warp_affine_u16(img, M))


def test_config2_slab_end_to_end(dev):
    """A 1080p slab shaped like BASELINE config 2 (ORB-like D=32, n_tpl=500, rigid):
    the recovered frame->template maps match the ground truth, RANSAC and the warp agree
    with the oracle on every frame (each frame with its own content), and the input
    frames are left untouched."""
    F, H, W = 48, 1080, 1920
    ks = synthetic.make_keypoints(F, 500, 32, (H, W), seed=7)
    host_frames = distinct_frames(synthetic.make_texture((H, W), seed=0), F)
    frames = torch.from_numpy(host_frames).to(dev)
    frames_before = frames.clone()
    inp = pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                              torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                              torch.from_numpy(ks.q_off).to(dev), ks.q_off)
    cfg = pipeline.AlignConfig(n_kp_global=100)
    res = pipeline.align_slab(inp, cfg, logger=logging.getLogger("test"), keep_intermediates=True)
    torch.cuda.synchronize()
    assert torch.equal(frames, frames_before), "the pipeline wrote into its input frames"
    assert res.skipped == [] and res.interpolated == []
    np.testing.assert_allclose(res.affines[:, :, :2], ks.gt[:, :, :2], atol=2e-3)
    np.testing.assert_allclose(res.affines[:, :, 2], ks.gt[:, :, 2], atol=0.5)
    # RANSAC parity on the device-gathered point lists
    kq = res.match.kp_ordered.cpu().numpy()
    inl = res.ransac.inliers.cpu().numpy().astype(bool)
    po, pi = res.consensus.pt_off, res.consensus.pt_idx
    best, n_in = res.ransac.best_trial.cpu().numpy(), res.ransac.n_inliers.cpu().numpy()
    for f in range(F):
        L = pi[po[f]:po[f + 1]]
        p, i_ref, bt, ni = oracle.ransac_rigid(kq[f][L], ks.kp_tpl[L])
        assert np.array_equal(inl[po[f]:po[f + 1]], i_ref), f
        assert best[f] == bt and n_in[f] == ni, f
        np.testing.assert_allclose(res.affines[f], p, rtol=1e-4, atol=1e-6)
    out = res.aligned.cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_affine_u16(host_frames[f], res.affines[f])), f


@pytest.mark.parametrize("beside", [False, True])
def test_overlapped_slabs_equal_align_slab(dev, beside):
    """OverlappedSlabs (kernel stream: [match(k)] -> warp(k-1); analysis stream: [match(k)]
    -> lookup + RANSAC(k) beside the warp; beside: the match on the analysis stream too)
    gives the same affines and warped frames as the sequential align_slab, leading,
    interior and trailing gaps included."""
    cfg = pipeline.AlignConfig(n_kp_global=60)
    slabs = _gap_slabs(dev)
    ref = [pipeline.align_slab(s, cfg) for s in slabs]
    ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=beside)
    _check_overlapped(ov, slabs, ref)


def _check_overlapped(ov, slabs, ref):
    got = [ov.submit(s) for s in slabs]
    assert got[0] is None
    got = got[1:] + ov.flush()
    assert ov.flush() == []
    ov.synchronize()
    assert [len(r.skipped) for r in ref] == [3, 4, 0]
    for r, g in zip(ref, got):
        assert np.array_equal(r.affines, g.affines, equal_nan=True)
        assert r.skipped == g.skipped and r.interpolated == g.interpolated
        assert torch.equal(r.aligned, g.aligned)


def _gap_slabs(dev):
    F, H, W = 24, 270, 480
    slabs = []
    for seed in (11, 12, 13):
        ks = synthetic.make_keypoints(F, 300, 32, (H, W), seed=seed)
        # frames whose descriptors are all one row pass no ratio test (d1 == d2), so they
        # get no model: leading, interior and trailing gaps (host interpolation, then a
        # second warp of those frames)
        rng = np.random.default_rng(seed)
        for f in {11: (0, 1, 7), 12: (9, 10, 11, F - 1), 13: ()}[seed]:
            a, b = ks.q_off[f], ks.q_off[f + 1]
            ks.des_q[a:b] = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        base = synthetic.make_texture((H, W), seed=seed)
        frames = torch.from_numpy(np.broadcast_to(base, (F, H, W)).copy()).to(dev)
        slabs.append(pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev),
                                         torch.from_numpy(ks.kp_tpl).to(dev), torch.from_numpy(ks.des_q).to(dev),
                                         torch.from_numpy(ks.kp_q).to(dev), torch.from_numpy(ks.q_off).to(dev),
                                         ks.q_off))
    return slabs


def test_device_lists_follow_the_seed_after_host_list_ransac(dev, caplog):
    """The device-list RANSAC (align_slab, OverlappedSlabs) re-installs its own seed's
    hypothesis tables when another call on the same context has replaced them (a host-list
    ransac_rigid with another RANDOM_SEED); OverlappedSlabs writes VA:279-283's low-count
    log lines from the point counts it copied with the parameters."""
    F, H, W = 16, 270, 480
    ks = synthetic.make_keypoints(F, 300, 32, (H, W), seed=21)
    for f in (2, 3):  # two frames without a model: low-count log lines
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ks.des_q[a:b] = ks.des_q[a]
    base = synthetic.make_texture((H, W), seed=21)
    frames = torch.from_numpy(np.broadcast_to(base, (F, H, W)).copy()).to(dev)
    inp = pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                              torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                              torch.from_numpy(ks.q_off).to(dev), ks.q_off)
    cfg42, cfg7 = pipeline.AlignConfig(n_kp_global=60), pipeline.AlignConfig(n_kp_global=60, seed=7)
    a42 = pipeline.align_slab(inp, cfg42, keep_intermediates=True)
    # a host-list RANSAC with seed 7 on the same device replaces the context's tables
    po, pi = a42.consensus.pt_off, a42.consensus.pt_idx
    kq = a42.match.kp_ordered.cpu().numpy()
    r7 = stages.ransac_rigid(a42.match.kp_ordered.view(-1, 2), inp.kp_tpl, torch.from_numpy(po).to(dev), po,
                             pt_idx=torch.from_numpy(pi if pi.size else np.zeros(1, np.int32)).to(dev),
                             src_frame_stride=300, seed=7)
    p7 = r7.params.cpu().numpy()
    b42 = pipeline.align_slab(inp, cfg42)
    assert np.array_equal(a42.affines, b42.affines, equal_nan=True)
    assert torch.equal(a42.aligned, b42.aligned)
    # and the device lists with seed 7 give the host-list seed-7 result and the oracle's
    a7 = pipeline.align_slab(inp, cfg7)
    ok = ~np.isnan(p7).any(axis=(1, 2))
    assert np.array_equal(a7.affines[ok], p7[ok])
    for f in np.flatnonzero(ok)[::5]:
        L = pi[po[f]:po[f + 1]]
        p, _, _, _ = oracle.ransac_rigid(kq[f][L], ks.kp_tpl[L], seed=7)
        np.testing.assert_allclose(a7.affines[f], p, rtol=1e-9, atol=1e-9)
    logger = logging.getLogger("test_seed_lists")
    n_low = int((np.diff(po) < cfg42.n_kp_frame_skip).sum())
    for beside in (False, True):
        caplog.clear()
        with caplog.at_level(logging.INFO, logger="test_seed_lists"):
            ov = pipeline.OverlappedSlabs(dev, cfg42, logger=logger, match_beside=beside)
            got = [r for r in (ov.submit(inp), ov.submit(inp)) if r is not None] + ov.flush()
            ov.synchronize()
        low = [r.getMessage() for r in caplog.records if "low keypoint count" in r.getMessage()]
        assert len(got) == 2 and n_low >= 2 and len(low) == 2 * n_low
        for g in got:
            assert np.array_equal(g.affines, a42.affines, equal_nan=True)


def test_euclidean_min_samples_other_than_two_raises(dev):
    F, H, W = 4, 96, 128
    ks = synthetic.make_keypoints(F, 64, 32, (H, W), seed=1)
    frames = torch.zeros((F, H, W), dtype=torch.uint16, device=dev)
    inp = pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                              torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                              torch.from_numpy(ks.q_off).to(dev), ks.q_off)
    with pytest.raises(ValueError, match="min_samples=2"):
        pipeline.align_slab(inp, pipeline.AlignConfig(n_kp_global=30, ransac_min_samples=3))


@pytest.mark.parametrize("model,rate,beside", [("euclidean", 2, True), ("euclidean", 3, False),
                                               ("projective", 1, False), ("projective", 1, True)])
def test_overlapped_slabs_host_maps_and_projective(dev, model, rate, beside):
    """The OverlappedSlabs paths test_overlapped_slabs_equal_align_slab does not reach:
    frame_downsample_rate > 1 (every full-rate frame's map comes from the host NaN-padding
    + interpolation, so the warp waits for the host; with corun the host waits for RANSAC
    on the analysis stream), and the projective model on device maps (warpPerspective of
    RANSAC's own [F, 3, 3] output, then the re-warp of model-less frames with the
    gap-filled homographies).  Equal to align_slab, gaps included."""
    S, H, W = 12, 180, 240
    cfg = pipeline.AlignConfig(n_kp_global=40, ransac_model=model, frame_downsample_rate=rate)
    slabs = []
    for k, seed in enumerate((41, 42, 43)):
        ks = synthetic.make_keypoints(S, 200, 32, (H, W), seed=seed, model=model)
        rng = np.random.default_rng(seed)
        for f in ((0, 5), (4, 5, S - 1), ())[k]:  # model-less sample frames (see above)
            a, b = ks.q_off[f], ks.q_off[f + 1]
            ks.des_q[a:b] = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        base = synthetic.make_texture((H, W), seed=seed)
        frames = torch.from_numpy(np.broadcast_to(base, (S * rate, H, W)).copy()).to(dev)
        slabs.append(pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev),
                                         torch.from_numpy(ks.kp_tpl).to(dev), torch.from_numpy(ks.des_q).to(dev),
                                         torch.from_numpy(ks.kp_q).to(dev), torch.from_numpy(ks.q_off).to(dev),
                                         ks.q_off))
    ref = [pipeline.align_slab(s, cfg) for s in slabs]
    assert [len(r.skipped) for r in ref] == [2, 3, 0]
    ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=beside)
    got = [ov.submit(s) for s in slabs]
    got = got[1:] + ov.flush()
    ov.synchronize()
    for r, g in zip(ref, got):
        assert r.affines.shape[0] == S * rate
        assert np.array_equal(r.affines, g.affines, equal_nan=True)
        assert r.skipped == g.skipped and r.interpolated == g.interpolated
        assert torch.equal(r.aligned, g.aligned)


def test_align_streamed_equals_device_resident(dev):
    """Host-resident frames streamed through the warp in slabs (3 streams, double
    buffering) give exactly the device-resident slab result."""
    from kcmc_amd import pipeline, synthetic

    F, H, W = 37, 96, 160
    ks = synthetic.make_keypoints(F, 120, 32, (H, W), seed=21)
    base = synthetic.make_texture((H, W), seed=22)
    frames = torch.from_numpy(np.broadcast_to(base, (F, H, W)).copy())
    inp = pipeline.SlabInputs(frames.to(dev), torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                              torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                              torch.from_numpy(ks.q_off).to(dev), ks.q_off)
    cfg = pipeline.AlignConfig(n_kp_global=40)
    ref = pipeline.align_slab(inp, cfg)
    out, res = pipeline.align_streamed(frames.pin_memory(), inp, cfg, slab=8)
    torch.cuda.synchronize()
    assert np.array_equal(out.numpy(), ref.aligned.cpu().numpy())
    assert np.array_equal(res.affines, ref.affines)


def test_align_images_with_gpu_orb_detector(dev):
    """align_images from raw uint16 frames with the build's GPU detector: normalisation,
    detection, matching, consensus, RANSAC and warp all on the device; the recovered
    translations are the synthetic jitter (integer shifts of a textured scene)."""
    rng = np.random.default_rng(31)
    H, W, F = 200, 260, 8
    lo = rng.integers(0, 60000, (H // 4 + 8, W // 4 + 8)).astype(np.float64)
    scene = np.clip(np.kron(lo, np.ones((4, 4))) + rng.normal(0, 800, (H + 32, W + 32)), 0, 65535).astype(np.uint16)
    shifts = [(int(a), int(b)) for a, b in rng.integers(-6, 7, (F, 2))]
    shifts[F // 2] = (0, 0)  # the template frame
    imgs = np.stack([scene[16 + dy:16 + dy + H, 16 + dx:16 + dx + W] for dy, dx in shifts])
    aligned, eu, skipped = VideoAligner().align_images(imgs, n_kp_global=60, detector_algorithm="orb", frame_rate=30)
    assert skipped == [] and aligned.shape == imgs.shape and aligned.dtype == np.uint16
    np.testing.assert_allclose(eu[:, 0], [dx for dy, dx in shifts], atol=1e-6)
    np.testing.assert_allclose(eu[:, 1], [dy for dy, dx in shifts], atol=1e-6)
    res = pipeline.align_frames(torch.from_numpy(imgs).to(dev), pipeline.AlignConfig(n_kp_global=60))
    assert np.array_equal(res.aligned.cpu().numpy(), aligned)
