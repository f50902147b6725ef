"""The drop-in VideoAligner over several devices in one process (kcmc_amd.multidevice).

On a one-GPU box the split is rehearsed with a repeated device: DEVICES = [0, 0] puts two
frame slabs on cuda:0, each with its own template copy, match, vote, lookup, RANSAC and
warp; the votes are merged once and the gaps interpolated once on the host.  The returned
arrays must equal DEVICES = [0] (one slab) exactly, with NaN gaps that cross the slab
boundary, temporal downsampling (frame_rate 200: rate 2), the extension models, host and
device inputs, and from raw frames with the GPU detector (normalisation over the split
stack)."""
import numpy as np
import pytest
import torch

from kcmc_amd import VideoAligner, stages, synthetic

pytestmark = pytest.mark.gpu


def _aligner(devices, model="euclidean"):
    class VA(VideoAligner):
        DEVICES = devices
        RANSAC_MODEL = model

    return VA()


def _keypoint_stack(n_sample, rate, model, blind, seed=61):
    H, W = 96, 160
    ks = synthetic.make_keypoints(n_sample, 150, 32, (H, W), seed=seed, model=model)
    rng = np.random.default_rng(seed)
    for f in blind:  # every descriptor one row: no match passes the ratio test (d1 == d2), no model
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ks.des_q[a:b] = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    base = synthetic.make_texture((H, W), seed=seed)
    frames = np.ascontiguousarray(np.stack([np.roll(base, (2 * f, 5 * f), axis=(0, 1))
                                            for f in range(n_sample * rate - rate // 2)]))
    kq = [ks.kp_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(n_sample)]
    dq = [ks.des_q[ks.q_off[f]:ks.q_off[f + 1]] for f in range(n_sample)]
    return ks, frames, kq, dq


@pytest.mark.parametrize("model,rate,blind", [("euclidean", 1, (5, 6, 7)), ("euclidean", 2, (4, 5)),
                                              ("affine", 1, (0, 1, 6)), ("euclidean", 1, (10, 11))])
def test_two_slabs_on_one_gpu_equal_one_slab(dev, model, rate, blind):
    n_sample = 12
    ks, frames, kq, dq = _keypoint_stack(n_sample, rate, model, blind)
    out = {}
    for devices in ([0], [0, 0], [0, 0, 0]):
        va = _aligner(devices, model)
        aligned, eu, skipped = va.align_keypoints(frames, ks.kp_tpl, ks.des_tpl, kq, dq, n_kp_global=40,
                                                  frame_rate=100 * rate)
        out[len(devices)] = (aligned, eu, skipped, va.interpolated_idxs)
    ref = out[1]
    assert isinstance(ref[0], np.ndarray) and ref[0].shape == frames.shape
    assert len(ref[2]) >= len(blind)  # the premise: frames without a model
    for k in (2, 3):
        np.testing.assert_array_equal(out[k][0], ref[0])
        np.testing.assert_array_equal(out[k][1], ref[1])
        assert out[k][2] == ref[2] and out[k][3] == ref[3]


def test_device_input_stays_on_device(dev):
    ks, frames, kq, dq = _keypoint_stack(9, 1, "euclidean", (4,))
    fr = torch.from_numpy(frames).to(dev)
    a1, e1, s1 = _aligner([0]).align_keypoints(fr, ks.kp_tpl, ks.des_tpl, kq, dq, n_kp_global=40)
    a2, e2, s2 = _aligner([0, 0]).align_keypoints(fr, ks.kp_tpl, ks.des_tpl, kq, dq, n_kp_global=40)
    assert isinstance(a2, torch.Tensor) and a2.device == fr.device
    assert torch.equal(a1, a2) and s1 == s2
    np.testing.assert_array_equal(e1, e2)


def test_brightest_px_over_parts_equals_whole(dev):
    rng = np.random.default_rng(9)
    x = rng.integers(0, 65536, (7, 33, 41)).astype(np.uint16)
    x[2, 3, 4] = 65535
    whole = torch.from_numpy(x).to(dev)
    parts = [whole[:3], whole[3:3], whole[3:]]
    b = stages.brightest_px(parts)
    assert b == stages.brightest_px(whole) == np.percentile(x, 99.99)
    # a slab that starts mid-allocation (3 frames of 33 x 41 u16 = 8118 bytes in): the
    # 16-byte kernels work on an aligned copy
    assert whole[3:].data_ptr() % 16 != 0
    np.testing.assert_array_equal(stages.max_scale_u8(whole[3:], b).cpu().numpy(), stages.max_scale_lut(b)[x[3:]])


def test_align_images_gpu_detector_split(dev):
    """align_images from raw uint16 frames with the GPU detector: the percentile of the
    split stack from the summed per-device histograms, detection per slab; identical to
    one slab."""
    rng = np.random.default_rng(31)
    H, W, F = 200, 260, 9
    lo = rng.integers(0, 60000, (H // 4 + 8, W // 4 + 8)).astype(np.float64)
    scene = np.clip(np.kron(lo, np.ones((4, 4))) + rng.normal(0, 800, (H + 32, W + 32)), 0, 65535).astype(np.uint16)
    shifts = [(int(a), int(b)) for a, b in rng.integers(-6, 7, (F, 2))]
    shifts[F // 2] = (0, 0)
    imgs = np.stack([scene[16 + dy:16 + dy + H, 16 + dx:16 + dx + W] for dy, dx in shifts])
    a1, e1, s1 = _aligner([0]).align_images(imgs, n_kp_global=60, detector_algorithm="orb", frame_rate=30)
    a2, e2, s2 = _aligner([0, 0]).align_images(imgs, n_kp_global=60, detector_algorithm="orb", frame_rate=30)
    assert s1 == s2 == []
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_allclose(e2[:, 0], [dx for dy, dx in shifts], atol=1e-6)
