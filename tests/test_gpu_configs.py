"""Parity of the HIP hot path at each BASELINE config's own sizes (configs c1, c3, c4, c5;
c2 is covered by test_gpu_kernels / test_gpu_pipeline and by bench.py).

Every check compares the path behind the C ABI with the CPU oracle on the same seeded
inputs (kcmc_amd.synthetic, the bench's generator):
  * K1 (VA:194-214): survivor bitmask and set order, best-match reorder, log counts;
  * consensus (VA:224-286): Counter order, votes and per-frame CPython set-order lists;
  * K2 (VA:288-323, skimage 0.18.3 ransac): winning trial, inlier mask, n_inliers, and
    parameters within 1e-6 relative (north_star: 1e-4);
  * K3 (VA:455-458): the warped frame bit-exact (north_star: 1 LSB).
Every frame of a slab has its own content (the base texture rolled by a per-frame
offset), so a tile that read another frame's (or another workgroup's) staged data cannot
reproduce the right value by accident; the warp is compared on every frame, and the
input frames are checked unchanged after the pipeline (a stray write into them would
show as a warp mismatch that the warp itself did not cause).  The matcher is compared
on every frame at c1/c3 and on 4 frames at c4/c5.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import distinct_frames
from kcmc_amd import pipeline, stages, synthetic

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _texture(H, W, C, seed):
    if C == 1:
        return synthetic.make_texture((H, W), seed=seed)
    return np.stack([synthetic.make_texture((H, W), seed=seed + c) for c in range(C)], axis=-1)


def _sets_from_bits(bits, n_tpl):
    out = []
    for row in bits:
        kept = [i for i in range(n_tpl) if (int(row[i >> 5]) >> (i & 31)) & 1]
        out.append(set(kept))  # built from an ascending list, like set(dist_matches) (VA:214)
    return out


def _oracle_match(ks, f, descriptor):
    a, b = ks.q_off[f], ks.q_off[f + 1]
    knn = oracle.knn2_l2f32 if descriptor == "f32" else oracle.knn2_l2u8
    idx, dist = knn(ks.des_tpl, ks.des_q[a:b])
    return oracle.filter_matches(idx, dist, ks.kp_tpl, ks.kp_q[a:b])


def _check_slab(dev, *, F, H, W, C, n_tpl, D, model, n_kp_global, descriptor="u8", seed=31, match_frames=None,
                ransac_frames=None):
    ks = synthetic.make_keypoints(F, n_tpl, D, (H, W), seed=seed, model=model, descriptor=descriptor)
    base = _texture(H, W, C, seed + 1)
    host_frames = distinct_frames(base, F)
    frames = _t(host_frames, dev)
    frames_before = frames.clone()
    inp = pipeline.SlabInputs(frames, _t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev),
                              _t(ks.kp_q, dev), _t(ks.q_off, dev), ks.q_off)
    cfg = pipeline.AlignConfig(n_kp_global=n_kp_global, ransac_model=model)
    res = pipeline.align_slab(inp, cfg, keep_intermediates=True)
    torch.cuda.synchronize()
    assert torch.equal(frames, frames_before), "the pipeline wrote into its input frames"
    del frames_before
    m, cons, rr = res.match, res.consensus, res.ransac
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kq = m.kp_ordered.cpu().numpy()
    counts = m.counts.cpu().numpy()
    gpu_sets = _sets_from_bits(bits, n_tpl)

    # K1 + filters against the oracle
    for f in (range(F) if match_frames is None else match_frames):
        s, kqo, cnt = _oracle_match(ks, f, descriptor)
        assert gpu_sets[f] == s, f
        assert list(gpu_sets[f]) == list(s), f  # CPython set order of the survivors
        assert np.array_equal(kq[f], kqo), f
        assert counts[f].tolist() == list(cnt), f
        assert len(s) > n_tpl // 3, (f, len(s))  # the synthetic frames match well

    # consensus against real CPython sets / Counter
    c_set, c_idx, c_votes = oracle.consensus(gpu_sets, n_kp_global)
    assert cons.order.tolist() == list(c_idx)
    assert cons.votes.tolist() == list(c_votes)
    lists = oracle.lookup(c_set, gpu_sets)
    po, pi = cons.pt_off, cons.pt_idx
    for f in range(F):
        assert pi[po[f]:po[f + 1]].tolist() == lists[f], f

    # K2 against the oracle on the same point lists
    inl = rr.inliers.cpu().numpy().astype(bool)
    n_in = rr.n_inliers.cpu().numpy()
    best = rr.best_trial.cpu().numpy()
    params = rr.params.cpu().numpy()
    n_fit = 0
    for f in (range(F) if ransac_frames is None else ransac_frames):
        L = pi[po[f]:po[f + 1]]
        if model == "euclidean":
            p, i_ref, bt, ni = oracle.ransac_rigid(kq[f][L], ks.kp_tpl[L])
        else:
            p, i_ref, bt, ni = oracle.ransac_model(kq[f][L], ks.kp_tpl[L], model)
            p = p[: params.shape[1]]
        assert best[f] == bt, f
        assert n_in[f] == ni, f
        assert np.array_equal(inl[po[f]:po[f + 1]], i_ref), f
        if not np.isnan(p).any():
            n_fit += 1
            np.testing.assert_allclose(params[f], p, rtol=1e-6, atol=1e-8, err_msg=str(f))
    assert n_fit > 0

    # K3: the warped frames bit-exact vs the oracle warp of the same maps
    out = res.aligned.cpu().numpy()
    warp = oracle.warp_perspective_u16 if model == "projective" else oracle.warp_affine_u16
    for f in range(F):
        ref = warp(host_frames[f], res.affines[f])
        bad = np.argwhere(out[f] != ref)
        # on a mismatch: where (the first positions, the values) and whether a second read
        # of the device buffer agrees with the first
        assert len(bad) == 0, (f, len(bad), bad[:16].tolist(), out[f][tuple(bad[:16].T)].tolist(),
                               ref[tuple(bad[:16].T)].tolist(),
                               bool(np.array_equal(res.aligned[f].cpu().numpy(), out[f])))
    return res, ks


def test_config1_512_akaze_rigid(dev):
    """c1: 512x512, n_tpl ~1000 AKAZE-sized (D = 61) descriptors, rigid RANSAC,
    n_kp_global 50 (the reference's own CPU-runnable case)."""
    res, ks = _check_slab(dev, F=16, H=512, W=512, C=1, n_tpl=1000, D=61, model="euclidean", n_kp_global=50)
    # the rigid fit recovers the ground-truth jitter
    np.testing.assert_allclose(res.affines[:, :, 2], ks.gt[:, :, 2], atol=1.0)


def test_config3_512_two_photon_affine(dev):
    """c3: 512x512, n_tpl 500, D = 61, affine RANSAC, n_kp_global 50."""
    _check_slab(dev, F=16, H=512, W=512, C=1, n_tpl=500, D=61, model="affine", n_kp_global=50, seed=37)


def test_config4_matcher_4096_keypoints(dev):
    """c4's matcher shape: 4096 template keypoints x ~4500 per frame, D = 61 (the
    16-workgroup template grid, 18 frame chunks of 256 rows)."""
    F = 6
    ks = synthetic.make_keypoints(F, 4096, 61, (2160, 3840), seed=41, model="affine")
    m = stages.match_frames(_t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev),
                            _t(ks.q_off, dev), ks.q_off)
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kq = m.kp_ordered.cpu().numpy()
    idx = m.idx.cpu().numpy()
    dist = m.dist.cpu().numpy()
    for f in (0, 2, 3, F - 1):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ri, rd = oracle.knn2_l2u8(ks.des_tpl, ks.des_q[a:b])
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f
        s, kqo, _ = oracle.filter_matches(ri, rd, ks.kp_tpl, ks.kp_q[a:b])
        assert _sets_from_bits(bits[f:f + 1], 4096)[0] == s
        assert np.array_equal(kq[f], kqo)


def test_config4_4k_rgb_affine_slab(dev):
    """c4 end to end: 2160x3840x3 u16 frames, n_tpl 4096, D = 61, affine RANSAC with
    n_kp_global 500 (RANSAC on up to 500 points), per-channel warp."""
    _check_slab(dev, F=4, H=2160, W=3840, C=3, n_tpl=4096, D=61, model="affine", n_kp_global=500, seed=43)


def test_config5_float_matcher_4096x128(dev):
    """c5's matcher shape: 4096 float32 template descriptors x ~4500 per frame, D = 128
    (bf16x3 MFMA candidates + exact fp64 re-rank), bit-exact indices and distances."""
    F = 4
    ks = synthetic.make_keypoints(F, 4096, 128, (1080, 1920), seed=47, model="projective", descriptor="f32")
    idx, dist = stages.knn2_l2u8(_t(ks.des_tpl, dev), _t(ks.des_q, dev), _t(ks.q_off, dev),
                                 int(np.diff(ks.q_off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f in range(F):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ri, rd = oracle.knn2_l2f32(ks.des_tpl, ks.des_q[a:b])
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


def test_config5_1080p_sift_homography_slab(dev):
    """c5 end to end: 1080p u16, float SIFT-style descriptors (n_tpl 4096, D = 128),
    homography RANSAC with n_kp_global 200, warpPerspective."""
    _check_slab(dev, F=4, H=1080, W=1920, C=1, n_tpl=4096, D=128, model="projective", n_kp_global=200,
                descriptor="f32", seed=53)
