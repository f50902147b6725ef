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
