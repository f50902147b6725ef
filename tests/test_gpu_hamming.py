"""The opt-in NORM_HAMMING matcher (csrc/match_hamming.hip) through the C ABI against the
oracle (kcmc_oracle_knn2_hamming): indices and bit counts bit-exact, ties to the lower
frame index, chunk boundaries, frames without rows, more than one template group, and
the VA:196-214 filters on top.  Not the reference's matcher (VA:194 is NORM_L2)."""
import numpy as np
import pytest
import torch

import oracle
from kcmc_amd import stages, synthetic

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _csr(lists):
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in lists])
    return off


@pytest.mark.parametrize("D", [1, 5, 32, 33, 61, 64])
def test_knn2_hamming_matches_oracle(dev, D):
    rng = np.random.default_rng(200 + D)
    n_tpl = 300  # two template groups of 256 lanes
    tpl = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    frames = []
    for n_q in (600, 2, 0, 257, 256, 31):
        q = rng.integers(0, 256, (n_q, D), dtype=np.uint8)
        if n_q > 10:
            q[: n_q // 3] = tpl[rng.integers(0, n_tpl, n_q // 3)]  # exact matches
            q[7] = q[3]  # duplicate rows: ties go to the lower index
            q[n_q - 1] = q[3]
        frames.append(q)
    off = _csr(frames)
    idx, dist = stages.knn2_hamming(_t(tpl, dev), _t(np.concatenate(frames), dev), _t(off, dev),
                                    int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    for f, q in enumerate(frames):
        ri, rd = oracle.knn2_hamming(tpl, q)
        assert np.array_equal(idx[f], ri), f
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), f


def test_match_frames_hamming_filters_vs_oracle(dev):
    """ORB-shaped frames (n_tpl 500, 32 B, ~550 rows) through match_frames(norm='hamming')."""
    ks = synthetic.make_keypoints(12, 500, 32, (1080, 1920), seed=9)
    m = stages.match_frames(_t(ks.des_tpl, dev), _t(ks.kp_tpl, dev), _t(ks.des_q, dev), _t(ks.kp_q, dev),
                            _t(ks.q_off, dev), ks.q_off, norm="hamming")
    bits = m.keep_bits.cpu().numpy().view(np.uint32)
    kqo = m.kp_ordered.cpu().numpy()
    counts = m.counts.cpu().numpy()
    for f in range(12):
        a, b = ks.q_off[f], ks.q_off[f + 1]
        idx, dist = oracle.knn2_hamming(ks.des_tpl, ks.des_q[a:b])
        s, kq, cnt = oracle.filter_matches(idx, dist, ks.kp_tpl, ks.kp_q[a:b])
        kept = [i for i in range(500) if (bits[f, i >> 5] >> (i & 31)) & 1]
        assert kept == sorted(s)
        assert np.array_equal(kqo[f], kq)
        assert counts[f].tolist() == list(cnt)


def test_hamming_rejects_float_descriptors(dev):
    d = torch.zeros((4, 8), dtype=torch.float32, device=dev)
    off = np.array([0, 4], np.int32)
    with pytest.raises(TypeError):
        stages.match_frames(d, torch.zeros((4, 2), dtype=torch.float64, device=dev), d,
                            torch.zeros((4, 2), dtype=torch.float64, device=dev), _t(off, dev), off, norm="hamming")
