"""Pin the oracle of the build's ORB-style detector (f1) with an independent
pure-Python restatement of its definition on small images.  OpenCV is absent from
this image, so parity vs cv2.ORB is unpinned; the definition is the build's."""
import math

import numpy as np

import oracle
from kcmc_amd import orb

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _img(seed, H=72, W=90):
    rng = np.random.default_rng(seed)
    lo = rng.integers(0, 256, (H // 4 + 2, W // 4 + 2)).astype(np.float64)
    img = np.kron(lo, np.ones((4, 4)))[:H, :W] + rng.normal(0, 12, (H, W))
    return np.clip(img, 0, 255).astype(np.uint8)


def fast_score_py(img, x, y):
    v = int(img[y, x])
    d = [int(img[y + dy, x + dx]) - v for dx, dy in CIRCLE]
    best = -1000
    for k in range(16):
        arc = [d[(k + m) % 16] for m in range(9)]
        best = max(best, min(arc), min(-e for e in arc))
    return best


def harris_py(img, x, y, k=0.04):
    I = img.astype(np.int64)
    a = b = c = 0
    for dy in range(-3, 4):
        for dx in range(-3, 4):
            qy, qx = y + dy, x + dx
            ix = (I[qy - 1, qx + 1] + 2 * I[qy, qx + 1] + I[qy + 1, qx + 1]) - (I[qy - 1, qx - 1] + 2 * I[qy, qx - 1] + I[qy + 1, qx - 1])
            iy = (I[qy + 1, qx - 1] + 2 * I[qy + 1, qx] + I[qy + 1, qx + 1]) - (I[qy - 1, qx - 1] + 2 * I[qy - 1, qx] + I[qy - 1, qx + 1])
            a += ix * ix
            b += iy * iy
            c += ix * iy
    s = float(a + b)
    return float(a * b - c * c) - k * (s * s)


def test_fast_score_and_harris_match_python():
    img = _img(1)
    H, W = img.shape
    L = oracle.lib()
    p = np.ascontiguousarray(img).ctypes.data_as(oracle.ctypes.c_void_p)
    for y in range(4, H - 4, 3):
        for x in range(4, W - 4, 5):
            assert L.kcmc_oracle_fast_score(p, W, x, y) == fast_score_py(img, x, y)
            assert L.kcmc_oracle_harris(p, W, x, y, 0.04) == harris_py(img, x, y)


def detect_py(img, n_features=500, threshold=20, k=0.04, edge=16):
    H, W = img.shape
    score = np.zeros((H, W), np.int64)
    for y in range(3, H - 3):
        for x in range(3, W - 3):
            s = fast_score_py(img, x, y)
            score[y, x] = s if s > threshold else 0
    cands = []
    for ty in range(0, H, 16):
        for tx in range(0, W, 64):
            for y in range(ty, min(ty + 16, H)):
                for x in range(tx, min(tx + 64, W)):
                    if not (edge <= y < H - edge and edge <= x < W - edge) or score[y, x] == 0:
                        continue
                    s = score[y, x]
                    ok = all(s > score[y + dy, x + dx] or (s == score[y + dy, x + dx] and (dy > 0 or (dy == 0 and dx > 0)))
                             for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy)
                    if ok:
                        cands.append((harris_py(img, x, y, k), x, y))
    if len(cands) > n_features:
        T = sorted((c[0] for c in cands), reverse=True)[n_features - 1]
        n_gt = sum(c[0] > T for c in cands)
        kept, ties = [], 0
        for c in cands:
            if c[0] > T:
                kept.append(c)
            elif c[0] == T and ties < n_features - n_gt:
                kept.append(c)
                ties += 1
        cands = kept
    pat, cs = orb.rotated_patterns(), orb.bin_edges()
    I = img.astype(np.int64)
    w = np.array([1, 4, 6, 4, 1])
    ww = np.outer(w, w)

    def sm(x, y):
        return (int((ww * I[y - 2:y + 3, x - 2:x + 3]).sum()) + 128) >> 8

    kps, des = [], []
    for _, x, y in cands:
        m10 = m01 = 0
        for dy in range(-15, 16):
            for dx in range(-15, 16):
                if dx * dx + dy * dy <= 225:
                    m10 += dx * int(I[y + dy, x + dx])
                    m01 += dy * int(I[y + dy, x + dx])
        if m10 == 0 and m01 == 0:
            b = 0
        else:
            b = math.floor(math.atan2(m01, m10) / 0.19634954084936207) & 31
            b1 = (b + 1) & 31
            if m01 * cs[b, 0] - m10 * cs[b, 1] < 0:
                b = (b + 31) & 31
            elif m01 * cs[b1, 0] - m10 * cs[b1, 1] >= 0:
                b = b1
        d = np.zeros(32, np.uint8)
        for i in range(256):
            (px, py), (qx, qy) = pat[b, 2 * i], pat[b, 2 * i + 1]
            if sm(x + px, y + py) < sm(x + qx, y + qy):
                d[i // 8] |= 1 << (i % 8)
        kps.append((x, y))
        des.append(d)
    return np.array(kps, np.float64).reshape(-1, 2), np.array(des, np.uint8).reshape(-1, 32)


def test_orb_oracle_matches_python_restatement():
    for seed, nf in ((2, 500), (3, 7)):
        img = _img(seed)
        kp, des = oracle.orb_detect(img, n_features=nf, pattern=orb.rotated_patterns(), bin_cs=orb.bin_edges())
        kp2, des2 = detect_py(img, n_features=nf)
        assert len(kp) > 3
        assert np.array_equal(kp, kp2) and np.array_equal(des, des2)


def test_pattern_tables():
    p = orb.brief_pattern()
    assert p.shape == (512, 2) and ((p ** 2).sum(1) <= 169).all()
    r = orb.rotated_patterns()
    assert r.shape == (32, 512, 2) and np.abs(r).max() <= 14
    assert np.array_equal(r, orb.rotated_patterns())  # deterministic
