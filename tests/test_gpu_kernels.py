"""Parity of the HIP kernels (called through the C ABI) with the CPU oracle and the
reference goldens.  Integer/index results must be bit-exact; RANSAC parameters
within 1e-4 relative (north_star; we observe ~1e-12); warped pixels bit-exact to the
oracle (north_star tolerance: 1 LSB)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import distinct_frames, load_golden
from kcmc_amd import stages, synthetic

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _csr(lists):
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    return off


# ------------------------------------------------------------------------ K1
@pytest.mark.parametrize("D", [1, 7, 31, 32, 33, 61, 64])
def test_knn2_matches_oracle(dev, D):
    rng = np.random.default_rng(D)
    n_tpl = 300
    tpl = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    frames = []
    for f in range(5):
        n_q = int(rng.integers(2, 700))
        q = rng.integers(0, 256, (n_q, D), dtype=np.uint8)
        q[: n_q // 3] = tpl[rng.integers(0, n_tpl, n_q // 3)]  # exact matches -> ties
        if n_q > 10:
            q[7] = q[3]
            q[9] = q[3]
        frames.append(q)
    off = _csr(frames)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames), dev), _t(off, dev), int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_l2u8(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


def test_knn2_wide_keys_and_edge_counts(dev):
    # n_q > 1024 with D = 64: ssd << 11 | j would not fit 32 bits; the kernel keys each
    # 256-row chunk locally and folds the chunks into a 64-bit top-2
    rng = np.random.default_rng(11)
    D, n_tpl = 64, 97
    tpl = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    frames = [rng.integers(0, 256, (n, D), dtype=np.uint8) for n in (1500, 2, 1, 0, 33)]
    frames[0][1400] = tpl[5]
    off = _csr(frames)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames), dev), _t(off, dev), 1500)
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_l2u8(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


@pytest.mark.parametrize("D", [32, 61, 64])
def test_knn2_chunk_boundaries_and_extreme_bytes(dev, D):
    # exact duplicates straddling the 256-row LDS chunks (ties must go to the lower
    # frame index across chunks), and all-0 / all-255 descriptors (SSD = D * 255^2, the
    # largest key; the int8 offsets -128 / 127 at both ends)
    rng = np.random.default_rng(100 + D)
    n_tpl = 70
    tpl = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    tpl[0] = 0
    tpl[1] = 255
    tpl[2, ::2] = 255
    tpl[2, 1::2] = 0
    q = rng.integers(0, 256, (800, D), dtype=np.uint8)
    for j in (255, 256, 511, 512, 799):
        q[j] = tpl[5]
    for j in (250, 300, 767, 768):
        q[j] = tpl[6]
    q[600] = 255
    q[601] = 0
    q2 = np.full((3, D), 255, np.uint8)  # every distance to tpl[0] is the maximum
    q2[1] = 0
    frames = [q, q2, q[:257], q[:256], q[:255]]
    off = _csr(frames)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(np.concatenate(frames), dev), _t(off, dev), 800)
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, fq in enumerate(frames):
        ri, rd = oracle.knn2_l2u8(tpl, fq)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


def test_knn2_template_larger_than_a_workgroup(dev):
    rng = np.random.default_rng(12)
    tpl = rng.integers(0, 256, (1100, 32), dtype=np.uint8)
    q = rng.integers(0, 256, (600, 32), dtype=np.uint8)
    off = np.array([0, 600], np.int32)
    idx, dist = stages.knn2_l2u8(_t(tpl, dev), _t(q, dev), _t(off, dev), 600)
    ri, rd = oracle.knn2_l2u8(tpl, q)
    assert np.array_equal(idx.cpu().numpy()[0], ri)
    assert np.array_equal(dist.cpu().numpy()[0], rd)


def _match_all(g, dev):
    qo = g["q_offsets"].astype(np.int32)
    return stages.match_frames(_t(g["des_template"], dev), _t(g["kp_template"], dev), _t(g["des_query"], dev),
                               _t(g["kp_query"], dev), _t(qo, dev), qo)


@pytest.mark.parametrize("name", ["match_golden_akaze.npz", "match_golden_orb.npz"])
def test_match_frames_vs_reference_golden(dev, name):
    g = load_golden(name)
    m = _match_all(g, dev)
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kq = m.kp_ordered.cpu().numpy()
    counts = m.counts.cpu().numpy()
    so = g["kp_idxs_offsets"]
    n_tpl = g["kp_template"].shape[0]
    for f in range(len(so) - 1):
        kept = [i for i in range(n_tpl) if (bits[f, i >> 5] >> (i & 31)) & 1]
        assert kept == g["kp_idxs"][so[f]:so[f + 1]].tolist(), f
        assert list(set(kept)) == g["kp_idxs_setorder"][so[f]:so[f + 1]].tolist()
        assert np.array_equal(kq[f], g["kp_query_ordered"][f]), f
        assert counts[f].tolist() == g["log_counts"][f].tolist(), f


def test_match_frames_vs_oracle_at_config2_size(dev):
    """1080p ORB-like: n_tpl 500, D 32, ~550 keypoints per frame."""
    ks = synthetic.make_keypoints(24, 500, 32, (1080, 1920), seed=5)
    m = stages.match_frames(_t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev),
                            _t(ks.q_off, dev), ks.q_off)
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kqo = m.kp_ordered.cpu().numpy()
    for f in range(24):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        idx, dist = oracle.knn2_l2u8(ks.des_tpl, ks.des_q[a:b])
        s, kq, cnt = oracle.filter_matches(idx, dist, ks.kp_tpl, ks.kp_q[a:b])
        kept = [i for i in range(500) if (bits[f, i >> 5] >> (i & 31)) & 1]
        assert kept == sorted(s)
        assert np.array_equal(kqo[f], kq)
        assert len(kept) > 200  # the synthetic data matches well


def test_match_frames_rejects_frames_with_fewer_than_two_keypoints(dev):
    tpl = np.zeros((4, 8), np.uint8)
    off = np.array([0, 3, 4], np.int32)
    with pytest.raises(ValueError):
        stages.match_frames(_t(tpl, dev), _t(np.zeros((4, 2)), dev), _t(np.zeros((4, 8), np.uint8), dev),
                            _t(np.zeros((4, 2)), dev), _t(off, dev), off)


# ------------------------------------------------------------------------ K2
def _ransac(dev, tpls, qs, rate=1.0, trials=1000):
    off = _csr(qs)
    r = stages.ransac_rigid(_t(np.concatenate(qs).reshape(-1, 2), dev), _t(np.concatenate(tpls).reshape(-1, 2), dev),
                            _t(off, dev), off, trials=trials, spatial_rate=rate)
    return off, r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool), r.n_inliers.cpu().numpy(), \
        r.best_trial.cpu().numpy()


def test_ransac_vs_reference_golden(dev):
    g = load_golden("ransac_golden.npz")
    off = g["offsets"]
    F = len(off) - 1
    tpls = [g["kp_template"][off[f]:off[f + 1]] for f in range(F)]
    qs = [g["kp_query"][off[f]:off[f + 1]] for f in range(F)]
    for rate in (1, 2):
        sel = [f for f in range(F) if g["spatial_rate"][f] == rate]
        _, params, inl, nin, _ = _ransac(dev, [tpls[f] for f in sel], [qs[f] for f in sel], rate=rate)
        o2 = _csr([qs[f] for f in sel])
        for k, f in enumerate(sel):
            ref = g["affine"][f]
            if np.isnan(ref).any():
                assert np.isnan(params[k]).all(), f
                continue
            np.testing.assert_allclose(params[k], ref, rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(params[k], ref, rtol=1e-9, atol=1e-9)
            assert np.array_equal(inl[o2[k]:o2[k + 1]], g["inliers"][off[f]:off[f + 1]]), f
            assert nin[k] == g["n_inliers"][f]


def test_ransac_bit_exact_selection_vs_oracle(dev):
    """Same hypotheses, same residual arithmetic -> identical inliers and winning trial,
    including N > 128 (numpy's recursive pairwise order)."""
    rng = np.random.default_rng(21)
    tpls, qs = [], []
    # 63 / 64 / 65: the one-wave staging and refit (N <= 128) hold points lane and lane + 64
    for N in [3, 4, 5, 8, 9, 50, 63, 64, 65, 100, 127, 128, 129, 136, 200, 255, 256, 257, 300, 500, 777, 1024, 2000]:
        tpl = rng.uniform(0, 1000, (N, 2))
        A = synthetic.rigid(rng.normal(0, 0.02), rng.normal(0, 5), rng.normal(0, 5))
        q = (tpl - A[:, 2]) @ A[:, :2] + rng.normal(0, rng.uniform(0.1, 1.5), (N, 2))
        out = rng.random(N) < rng.uniform(0, 0.6)
        q[out] = rng.uniform(0, 1000, (int(out.sum()), 2))
        tpls.append(tpl.astype(np.float32).astype(np.float64))
        qs.append(q.astype(np.float32).astype(np.float64))
    off, params, inl, nin, best = _ransac(dev, tpls, qs)
    for f in range(len(qs)):
        p, i_ref, bt, ni = oracle.ransac_rigid(qs[f], tpls[f])
        assert best[f] == bt, f
        assert nin[f] == ni, f
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), f
        np.testing.assert_allclose(params[f], p, rtol=1e-10, atol=1e-10)


def test_ransac_degenerate_and_skipped_frames(dev):
    rng = np.random.default_rng(22)
    tpl = rng.uniform(0, 100, (10, 2))
    same = np.repeat(tpl[:1], 10, 0)  # all frame points identical -> every hypothesis degenerate
    off, params, inl, nin, best = _ransac(dev, [tpl, tpl[:2], tpl[:0], tpl], [same, tpl[:2] + 1, tpl[:0], tpl + 3])
    assert np.isnan(params[0]).all() and nin[0] == 0 and best[0] == -1
    assert np.isnan(params[1]).all() and np.isnan(params[2]).all()  # N < N_KP_FRAME_SKIP
    np.testing.assert_allclose(params[3], [[1, 0, -3], [0, 1, -3]], atol=1e-9)


def test_ransac_exact_data_early_exit(dev):
    # integer points + integer translation: every residual is exactly 0 -> S == 0 at trial 0
    tpl = np.array([[x, y] for x in range(0, 50, 7) for y in range(0, 40, 9)], np.float64)
    q = tpl - np.array([4.0, -2.0])
    off, params, inl, nin, best = _ransac(dev, [tpl], [q])
    _, _, bt, ni = oracle.ransac_rigid(q, tpl)
    assert best[0] == bt == 0 and nin[0] == ni == len(tpl)
    np.testing.assert_allclose(params[0], [[1, 0, 4], [0, 1, -2]], atol=1e-12)


@pytest.mark.parametrize("thresh", [2.0, 1.7, 0.3])
def test_ransac_inlier_threshold_boundary(dev, thresh):
    """The count pass tests q = dx^2 + dy^2 < Tq instead of sqrt(q) < t: residuals within
    a few ulps of the threshold (both sides, exactly on it) give the oracle's inliers."""
    rng = np.random.default_rng(int(thresh * 10))
    tpl = rng.uniform(-3, 3, (60, 2))
    shift = np.array([0.75, -0.5])
    q = tpl - shift
    ang = rng.uniform(0, 2 * np.pi, 24)
    for k in range(24):  # |residual| = thresh * (1 + j * 2^-50), j in -3..3, and exact multiples
        rad = thresh * (1 + (k % 7 - 3) * 2.0 ** -50) if k < 21 else thresh
        d = np.array([np.cos(ang[k]), np.sin(ang[k])]) * rad if k < 21 else np.array([rad, 0.0])
        q[k] = tpl[k] - shift - d
    off = _csr([q])
    r = stages.ransac_rigid(_t(q, dev), _t(tpl, dev), _t(off, dev), off, residual_threshold=thresh)
    p, i_ref, bt, ni = oracle.ransac_rigid(q, tpl, thresh=thresh)
    assert r.best_trial.cpu().numpy()[0] == bt
    assert r.n_inliers.cpu().numpy()[0] == ni
    assert np.array_equal(r.inliers.cpu().numpy().astype(bool), i_ref)
    np.testing.assert_allclose(r.params.cpu().numpy()[0], p, rtol=1e-10, atol=1e-10)
    assert 36 <= ni < 60


@pytest.mark.parametrize("thresh", [2.0, 1e-120, 5e-5])
def test_ransac_two_phase_ties_and_exact_fallback(dev, thresh):
    """Phase A (counts through q < tq, fp32 S estimates) hands phase B every trial whose S
    can tie the best: near-ties (a nearly noise-free inlier set: many two-point models
    with S within 1e-9 relative), exact ties (duplicated points give identical models:
    the lower trial wins), N > 128 (the wave-evaluated pairwise plan) -- and the frames it
    cannot certify fall back to exact scoring: a threshold whose tq is outside the range
    (1e-120), no trial with inliers (5e-5 on noisy data), exact data (S == 0)."""
    rng = np.random.default_rng(int(-np.log10(thresh)) + 31)
    tpls, qs = [], []
    for N, noise in [(40, 1e-9), (90, 1e-6), (90, 0.3), (150, 1e-7), (300, 0.5), (12, 0.0)]:
        tpl = rng.uniform(0, 1000, (N, 2))
        A = synthetic.rigid(rng.normal(0, 0.02), rng.normal(0, 5), rng.normal(0, 5))
        q = (tpl - A[:, 2]) @ A[:, :2] + rng.normal(0, noise, (N, 2)) if noise else tpl - np.array([3.0, 1.0])
        if N == 90 and noise == 0.3:  # duplicates: swapped / repeated pairs fit identical models
            q[45:], tpl[45:] = q[:45], tpl[:45]
        tpls.append(tpl)
        qs.append(q)
    off, params, inl, nin, best = _ransac_t(dev, tpls, qs, thresh)
    for f in range(len(qs)):
        p, i_ref, bt, ni = oracle.ransac_rigid(qs[f], tpls[f], thresh=thresh)
        assert best[f] == bt, f
        assert nin[f] == ni, f
        assert np.array_equal(inl[off[f]:off[f + 1]], i_ref), f
        np.testing.assert_allclose(params[f], p, rtol=1e-10, atol=1e-10, equal_nan=True)


def _ransac_t(dev, tpls, qs, thresh):
    off = _csr(qs)
    r = stages.ransac_rigid(_t(np.concatenate(qs).reshape(-1, 2), dev), _t(np.concatenate(tpls).reshape(-1, 2), dev),
                            _t(off, dev), off, residual_threshold=thresh)
    return off, r.params.cpu().numpy(), r.inliers.cpu().numpy().astype(bool), r.n_inliers.cpu().numpy(), \
        r.best_trial.cpu().numpy()


def test_ransac_gather_mode_matches_contiguous(dev):
    rng = np.random.default_rng(23)
    n_tpl, F = 60, 7
    kp_tpl = rng.uniform(0, 500, (n_tpl, 2))
    kp_ord = kp_tpl[None] + rng.normal(0, 0.5, (F, n_tpl, 2)) + 2.0
    lists = [rng.permutation(n_tpl)[: int(rng.integers(0, 40))].astype(np.int32) for _ in range(F)]
    off = _csr(lists)
    r = stages.ransac_rigid(_t(kp_ord.reshape(-1, 2), dev), _t(kp_tpl, dev), _t(off, dev), off,
                            pt_idx=_t(np.concatenate(lists), dev), src_frame_stride=n_tpl)
    _, p2, _, _, _ = _ransac(dev, [kp_tpl[L] for L in lists], [kp_ord[f][L] for f, L in enumerate(lists)])
    np.testing.assert_array_equal(r.params.cpu().numpy(), p2)


# ------------------------------------------------------------------------ K3
@pytest.mark.parametrize("shape", [(1, 5, 7), (3, 64, 128), (2, 67, 131), (2, 130, 257), (2, 90, 200), (1, 57, 136),
                                   (1, 1080, 1920)])
def test_warp_matches_oracle(dev, shape):
    F, H, W = shape
    rng = np.random.default_rng(H * W)
    imgs = rng.integers(0, 65536, shape).astype(np.uint16)
    Ms = []
    for f in range(F):
        A = synthetic.rigid(rng.normal(0, 0.03), rng.normal(0, 6), rng.normal(0, 6))
        if f % 3 == 1:
            A[:, :2] *= 1.05
        Ms.append(A)
    Ms = np.stack(Ms)
    out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f])), f


def test_warp_stream_workspace_reuse(dev):
    """The per-stream cached workspace (kcmc_ctx::stream_ws): back-to-back warps of
    growing and shrinking tile counts queued on two streams without host syncs (the
    cache is reused in stream order, replaced by a larger block, never shared across
    streams) give the same pixels as one warp at a time."""
    rng = np.random.default_rng(21)
    sizes = [(2, 270, 480), (6, 540, 960), (1, 135, 240), (4, 540, 960), (3, 1080, 1920)]
    jobs = []
    for F, H, W in sizes:
        imgs = rng.integers(0, 65536, (F, H, W)).astype(np.uint16)
        Ms = np.stack([synthetic.rigid(rng.normal(0, 0.01), rng.normal(0, 4), rng.normal(0, 4)) for _ in range(F)])
        jobs.append((_t(imgs, dev), _t(Ms, dev)))
    ref = [stages.warp_affine_u16(i, m).cpu() for i, m in jobs]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    # every (rep, job) has its own output: the two streams run concurrently with no
    # cross-stream waits between jobs, so a cache shared across streams would race
    outs = [[torch.zeros_like(i) for i, _ in jobs] for _ in range(3)]
    cur = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(cur)
    for rep in range(3):
        for k, (i, m) in enumerate(jobs):
            s = streams[(k + rep) % 2]
            with torch.cuda.stream(s):
                stages.warp_affine_u16(i, m, out=outs[rep][k])
    for s in streams:
        cur.wait_stream(s)
    torch.cuda.synchronize(dev)
    for rep in range(3):
        for k in range(len(jobs)):
            assert torch.equal(outs[rep][k].cpu(), ref[k]), (rep, k)


def test_warp_graph_capture_replay_after_larger_eager_warp(dev):
    """A warp captured into a hipGraph owns its workspace: replaying the graph after a
    larger eager warp on the same stream (which replaces that stream's cached block)
    still gives the captured warp's pixels."""
    rng = np.random.default_rng(23)
    small = _t(rng.integers(0, 65536, (2, 270, 480)).astype(np.uint16), dev)
    big = _t(rng.integers(0, 65536, (3, 1080, 1920)).astype(np.uint16), dev)
    Ms = _t(np.stack([synthetic.rigid(0.01, 2.5, -1.5), synthetic.rigid(-0.02, -3.0, 4.0)]), dev)
    Mb = _t(np.stack([synthetic.rigid(0.005 * k, 1.0 + k, -2.0) for k in range(3)]), dev)
    ref_small = stages.warp_affine_u16(small, Ms).cpu()
    ref_big = stages.warp_affine_u16(big, Mb).cpu()
    out_small = torch.zeros_like(small)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        stages.warp_affine_u16(small, Ms, out=out_small)  # eager warm-up: the stream's cached block
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        stages.warp_affine_u16(small, Ms, out=out_small)
    out_big = torch.zeros_like(big)
    with torch.cuda.stream(s):
        stages.warp_affine_u16(big, Mb, out=out_big)  # a larger block replaces the cache
        out_small.zero_()
        g.replay()
    torch.cuda.synchronize(dev)
    assert torch.equal(out_big.cpu(), ref_big)
    assert torch.equal(out_small.cpu(), ref_small)


@pytest.mark.parametrize("values", ["14bit", "hot", "blobs", "edge16384", "dense_hot", "bright_lines"])
def test_warp_fast_path_value_ranges(dev, values):
    # the fixed-pitch staged path picks its blend per tile: exact integer for boxes below
    # 16384, packed-fp32 OpenCV evaluation otherwise; mix both within one frame
    F, H, W = 3, 240, 512
    rng = np.random.default_rng(77)
    if values == "14bit":
        imgs = rng.integers(0, 16384, (F, H, W))
    elif values == "hot":  # isolated bright pixels: the per-row mixed blend
        imgs = rng.integers(0, 16384, (F, H, W))
        imgs[rng.random((F, H, W)) < 2e-4] = 65535
    elif values == "blobs":
        imgs = rng.integers(0, 8192, (F, H, W))
        blk = rng.random((F, H // 32 + 1, W // 32 + 1)) < 0.15
        imgs = np.where(np.repeat(np.repeat(blk, 32, 1), 32, 2)[:, :H, :W], imgs + 36000, imgs)
    elif values == "dense_hot":  # ~3 % hot pixels: many queued fix-ups per wave (queue flushes)
        imgs = rng.integers(0, 8192, (F, H, W))
        imgs[rng.random((F, H, W)) < 0.03] = 60000
    elif values == "bright_lines":  # bright horizontal lines: rows re-blended in float at once
        imgs = rng.integers(0, 8192, (F, H, W))
        imgs[:, 17::41, :] = 50000
        imgs[rng.random((F, H, W)) < 1e-3] = 65535
    else:  # straddle the 2^24 boundary of the integer blend sum
        imgs = rng.integers(16370, 16400, (F, H, W))
    imgs = imgs.astype(np.uint16)
    Ms = np.stack([synthetic.rigid(rng.normal(0, 0.02), rng.normal(0, 5), rng.normal(0, 5)) for _ in range(F)])
    out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f])), f


def test_warp_identity_inverse_map_and_extreme_maps(dev):
    rng = np.random.default_rng(31)
    imgs = rng.integers(0, 65536, (4, 33, 45)).astype(np.uint16)
    Ms = np.stack([np.array([[1.0, 0, 0], [0, 1, 0]]), np.array([[0.0, -1, 40], [1, 0, -3]]),
                   np.array([[3.0, 0.2, -50], [0.1, 0.2, 7]]), np.array([[1.0, 0, 1000], [0, 1, -1000]])])
    for inv in (False, True):
        out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev), inverse_map=inv).cpu().numpy()
        for f in range(4):
            assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f], inverse_map=inv)), (f, inv)
    assert np.array_equal(out[0], imgs[0])


@pytest.mark.parametrize("C,shape", [(3, (3, 240, 512)), (4, (2, 250, 520)), (3, (2, 250, 520))])
@pytest.mark.parametrize("values", ["14bit", "hot", "blobs", "full"])
def test_warp_multichannel_fast_path_value_ranges(dev, C, shape, values):
    """The planar fast path of C = 3 / 4 (boxes de-interleaved into channel planes at the
    fixed pitch, one b96 / b128 store per lane and row): dark, per-row mixed and bright
    blends, whole and partial tiles (W = 520, H = 250), near-identity maps."""
    F, H, W = shape
    rng = np.random.default_rng(C * 1000 + H)
    if values == "14bit":
        imgs = rng.integers(0, 16384, (F, H, W, C))
    elif values == "hot":
        imgs = rng.integers(0, 16384, (F, H, W, C))
        imgs[rng.random((F, H, W, C)) < 2e-4] = 65535
    elif values == "blobs":
        imgs = rng.integers(0, 8192, (F, H, W, C))
        blk = rng.random((F, H // 32 + 1, W // 32 + 1, 1)) < 0.15
        imgs = np.where(np.repeat(np.repeat(blk, 32, 1), 32, 2)[:, :H, :W], imgs + 36000, imgs)
    else:
        imgs = rng.integers(0, 65536, (F, H, W, C))
    imgs = imgs.astype(np.uint16)
    Ms = np.stack([synthetic.rigid(rng.normal(0, 0.02), rng.normal(0, 5), rng.normal(0, 5)) for _ in range(F)])
    out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f])), f


@pytest.mark.parametrize("C", [3, 4])
def test_warp_multichannel(dev, C):
    rng = np.random.default_rng(C)
    imgs = rng.integers(0, 65536, (2, 50, 70, C)).astype(np.uint16)
    Ms = np.stack([synthetic.rigid(0.02, 1.5, -2.25), synthetic.rigid(-0.01, -3.3, 0.7)])
    out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(2):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f]))


def test_warp_all_tile_paths_at_1080p(dev):
    """Rotations/zooms that put tiles on every path: LDS-staged boxes, boxes too large
    for LDS (direct gather), and boxes entirely outside the frame (zeros)."""
    rng = np.random.default_rng(41)
    H, W = 1080, 1920
    img = rng.integers(0, 65536, (H, W)).astype(np.uint16)
    Ms = [synthetic.rigid(np.deg2rad(6.0), 10.5, -7.25), synthetic.rigid(np.deg2rad(-30.0), 300, 100),
          np.array([[0.6, 0.01, 5.0], [-0.01, 0.6, 3.0]]), np.array([[1.8, 0.0, -400.0], [0.0, 1.8, -300.0]]),
          synthetic.rigid(0.0, 1500.0, 0.0)]
    imgs = distinct_frames(img, len(Ms))
    out = stages.warp_affine_u16(_t(imgs, dev), _t(np.stack(Ms), dev)).cpu().numpy()
    for f, M in enumerate(Ms):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], M)), f


@pytest.mark.parametrize("values", ["full", "14bit", "hot"])
def test_warp_64_row_tiles(dev, values):
    """Frame heights that are multiples of 64 but not of 56 (512 x 512: BASELINE config 3)
    take 64-row tiles: the fixed-pitch fast path for small rotations, the general staged
    path / direct gather / zeros for larger rotations, zooms and shifts off the frame."""
    rng = np.random.default_rng(64)
    H, W = 512, 512
    if values == "full":
        img = rng.integers(0, 65536, (H, W))
    elif values == "14bit":
        img = rng.integers(0, 16384, (H, W))
    else:
        img = rng.integers(0, 16384, (H, W))
        img[rng.random((H, W)) < 3e-4] = 65535
    img = img.astype(np.uint16)
    Ms = [synthetic.rigid(np.deg2rad(0.5), 3.25, -2.5), synthetic.rigid(np.deg2rad(2.4), -4.0, 1.75),
          synthetic.rigid(np.deg2rad(6.0), 10.5, -7.25), synthetic.rigid(np.deg2rad(-30.0), 100, 50),
          np.array([[0.6, 0.01, 5.0], [-0.01, 0.6, 3.0]]), np.array([[1.02, 0.0, -3.0], [0.0, 0.98, 2.0]]),
          synthetic.rigid(0.0, 900.0, 0.0), synthetic.rigid(0.0, 0.0, 0.0)]
    imgs = distinct_frames(img, len(Ms))
    out = stages.warp_affine_u16(_t(imgs, dev), _t(np.stack(Ms), dev)).cpu().numpy()
    for f, M in enumerate(Ms):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], M)), f


def test_warp_nan_map_gives_zeros(dev):
    """A frame without a RANSAC model (NaN map) warps to zeros (coordinates outside the
    image under BORDER_CONSTANT); the pipeline re-warps it with the gap-filled map."""
    rng = np.random.default_rng(5)
    img = rng.integers(1, 65536, (64, 136)).astype(np.uint16)
    fr = torch.from_numpy(np.broadcast_to(img, (3, 64, 136)).copy()).to(dev)
    M = np.stack([synthetic.rigid(0.01, 1.5, -2.0)] * 3)
    M[1, 0, 2] = np.nan
    for persp in (False, True):
        if persp:
            Mp = np.concatenate([M, np.tile([[[0.0, 0.0, 1.0]]], (3, 1, 1))], axis=1)
            out = stages.warp_perspective_u16(fr, _t(Mp, dev)).cpu().numpy()
        else:
            out = stages.warp_affine_u16(fr, _t(M, dev)).cpu().numpy()
        assert not out[1].any()
        assert out[0].any() and np.array_equal(out[0], out[2])


@pytest.mark.parametrize("shape", [(3, 120, 256, 3), (2, 96, 136, 4), (1, 2160, 3840, 3)])
def test_warp_multichannel_vector_staging(dev, shape):
    """C = 3 / 4 with W % 8 == 0: 16-byte staging of interleaved rows into 128 x 24
    tiles (and, at 4K, tiles on every path)."""
    rng = np.random.default_rng(shape[1])
    imgs = rng.integers(0, 65536, shape).astype(np.uint16)
    F = shape[0]
    Ms = [synthetic.rigid(np.deg2rad(0.4), 3.7, -2.2), synthetic.rigid(np.deg2rad(-25.0), 40.0, 10.0),
          np.array([[1.6, 0.02, -30.0], [0.01, 1.6, -20.0]])][:F]
    Ms = np.stack(Ms)
    out = stages.warp_affine_u16(_t(imgs, dev), _t(Ms, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], oracle.warp_affine_u16(imgs[f], Ms[f])), f
    Hs = np.concatenate([Ms, np.tile([[[0.0, 0.0, 1.0]]], (F, 1, 1))], axis=1)
    Hs[:, 2, :2] = [2e-5, -1e-5]
    outp = stages.warp_perspective_u16(_t(imgs, dev), _t(Hs, dev)).cpu().numpy()
    for f in range(F):
        assert np.array_equal(outp[f], oracle.warp_perspective_u16(imgs[f], Hs[f])), f
