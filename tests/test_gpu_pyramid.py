"""f4: the device pyrDown (csrc/pyramid.hip) against the C oracle, and the downsampled
align_images path (VA:105-108, VA:494-506) end to end."""
import numpy as np
import pytest
import torch

import oracle
from kcmc_amd import VideoAligner, pipeline, stages
from kcmc_amd.video_aligner import LoResVideoAligner

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(1, 1, 1), (2, 5, 7), (3, 64, 64), (2, 67, 131), (2, 130, 258), (1, 512, 512),
                                   (1, 1080, 1920), (2, 33, 4)])
def test_pyr_down_matches_oracle(dev, shape):
    F, H, W = shape
    rng = np.random.default_rng(H * 7 + W)
    imgs = rng.integers(0, 256, shape).astype(np.uint8)
    t = torch.from_numpy(imgs).to(dev)
    sizes = {((W + 1) // 2, (H + 1) // 2), (max(1, W // 2), max(1, H // 2))}
    if W % 2 == 1 and H % 2 == 1:
        sizes.add(((W + 2) // 2 + 0, (H + 2) // 2 + 0))
    for dw, dh in sorted(sizes):
        if abs(2 * dw - W) > 2 or abs(2 * dh - H) > 2:
            continue
        out = stages.pyr_down_u8(t, (dw, dh)).cpu().numpy()
        assert out.shape == (F, dh, dw)
        for f in range(F):
            np.testing.assert_array_equal(out[f], oracle.pyr_down_u8(imgs[f], (dw, dh)), err_msg=f"{(dw, dh)} {f}")


def test_pyr_down_size_assertion(dev):
    t = torch.zeros((2, 10, 20), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        stages.pyr_down_u8(t, (10, 20))  # VA:501 with spatial rate 1: dstsize = shape
    with pytest.raises(ValueError):
        stages.pyr_down_u8(t, (5, 10))  # (H//2, W//2) read as (width, height)
    assert stages.pyr_down_u8(t).shape == (2, 5, 10)


def test_downsample_u8_reference_quirks(dev):
    rng = np.random.default_rng(3)
    sq = torch.from_numpy(rng.integers(0, 256, (6, 48, 48)).astype(np.uint8)).to(dev)
    tpl = sq[2:3].contiguous()
    s, t = pipeline.downsample_u8(sq, tpl, 1, 2)  # rate 1: no pyrDown even at spatial rate 2
    assert s.shape == (6, 48, 48) and t.shape == (1, 48, 48)
    s, t = pipeline.downsample_u8(sq, tpl, 2, 2)
    assert s.shape == (3, 24, 24) and t.shape == (1, 24, 24)
    ref = [oracle.pyr_down_u8(f, (24, 24)) for f in sq.cpu().numpy()[::2]]
    np.testing.assert_array_equal(s.cpu().numpy(), np.stack(ref))
    rect = torch.zeros((4, 40, 60), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        pipeline.downsample_u8(rect, rect[:1].contiguous(), 2, 2)  # non-square: cv2.error in the reference
    with pytest.raises(ValueError):
        pipeline.downsample_u8(sq, tpl, 2, 1)  # base class at frame_rate >= 200


def _scene(rng, H, W, pad=32):
    lo = rng.integers(0, 60000, (H // 8 + 10, W // 8 + 10)).astype(np.float64)
    hi = np.kron(lo, np.ones((8, 8)))[: H + 2 * pad, : W + 2 * pad]
    return np.clip(hi + rng.normal(0, 800, hi.shape), 0, 65535).astype(np.uint16)


def test_lores_aligner_downsampled_path(dev):
    """LoResVideoAligner at frame_rate 200: every 2nd frame, pyrDown to half size on the
    device, GPU detection, RANSAC on half-resolution points with translations scaled by
    2 (VA:320); even shifts are recovered exactly on the sample frames, the others are
    the linear interpolation of their neighbours (VA:347-407)."""
    rng = np.random.default_rng(11)
    H = W = 256
    F = 9
    scene = _scene(rng, H, W)
    shifts = [(2 * int(a), 2 * int(b)) for a, b in rng.integers(-4, 5, (F, 2))]
    shifts[F // 2] = (0, 0)
    imgs = np.stack([scene[32 + dy:32 + dy + H, 32 + dx:32 + dx + W] for dy, dx in shifts])
    aligned, eu, skipped = LoResVideoAligner().align_images(imgs, n_kp_global=60, detector_algorithm="orb",
                                                            frame_rate=200)
    assert aligned.shape == imgs.shape and skipped == []
    for f in range(0, F, 2):
        np.testing.assert_allclose(eu[f, :2], [shifts[f][1], shifts[f][0]], atol=1e-6, err_msg=str(f))
    for f in range(1, F - 1, 2):
        np.testing.assert_allclose(eu[f, :2], (eu[f - 1, :2] + eu[f + 1, :2]) / 2, atol=1e-9)


def test_base_aligner_high_frame_rate_raises_like_reference(dev):
    rng = np.random.default_rng(5)
    imgs = _scene(rng, 64, 64)[None, :64, :64].repeat(4, 0)
    with pytest.raises(ValueError):
        VideoAligner().align_images(imgs, n_kp_global=20, detector_algorithm="orb", frame_rate=200)
