"""f4: the C oracle's cv2.pyrDown (oracle/kcmc_oracle.c kcmc_oracle_pyr_down_u8) pinned
against a pure-Python restatement that follows OpenCV 4.x pyrDown_ step by step
(imgproc/src/pyramids.cpp: tabL/tabR border columns, width0, the 5-row ring buffer of
horizontal sums, FixPtCast<uchar, 8>).  OpenCV itself is absent from this image, so
parity against cv2 is unpinned; these tests pin the oracle's closed form to OpenCV's
algorithm as restated, plus known answers.  The restatement steps through tabR two
source columns per output pixel (the closed form); that only matters for an even W with
dstsize.width = W/2 + 1, which the reference (dstsize = shape // 2) never requests."""
import numpy as np
import pytest

import oracle


def _border_reflect_101(p, n):
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p if p < 0 else n - 1 - (p - n) - 1
    return p


def _pyr_down_opencv_steps(src, dw, dh):
    """pyrDown_<FixPtCast<uchar, 8>> for one channel, as structured in OpenCV."""
    H, W = src.shape
    assert abs(dw * 2 - W) <= 2 and abs(dh * 2 - H) <= 2
    PD = 5
    width0 = min((W - PD // 2 - 1) // 2 + 1, dw)
    tabL = [_border_reflect_101(x - PD // 2, W) for x in range(PD + 2)]
    tabR = [_border_reflect_101(x + width0 * 2 - PD // 2, W) for x in range(PD + 2)]
    ring = {}
    sy0 = -(PD // 2)
    sy = sy0
    out = np.zeros((dh, dw), np.uint8)
    for y in range(dh):
        while sy <= 2 * y + 2:
            row = src[_border_reflect_101(sy, H)].astype(np.int64)
            buf = [0] * dw
            x = 0
            buf[0] = row[tabL[2]] * 6 + (row[tabL[1]] + row[tabL[3]]) * 4 + row[tabL[0]] + row[tabL[4]]
            x = 1
            if x < dw:
                while x < width0:
                    buf[x] = row[2 * x] * 6 + (row[2 * x - 1] + row[2 * x + 1]) * 4 + row[2 * x - 2] + row[2 * x + 2]
                    x += 1
                x_ = 0  # tabR column offset of the output pixel: 2 source columns per output
                while x < dw:
                    buf[x] = (row[tabR[x_ + 2]] * 6 + (row[tabR[x_ + 1]] + row[tabR[x_ + 3]]) * 4 + row[tabR[x_]]
                              + row[tabR[x_ + 4]])
                    x += 1
                    x_ += 2
            ring[(sy - sy0) % PD] = buf
            sy += 1
        rows = [ring[(2 * y - PD // 2 + k - sy0) % PD] for k in range(PD)]
        for x in range(dw):
            v = rows[2][x] * 6 + (rows[1][x] + rows[3][x]) * 4 + rows[0][x] + rows[4][x]
            out[y, x] = min(255, (v + 128) >> 8)
    return out


@pytest.mark.parametrize("shape", [(1, 1), (1, 2), (2, 1), (3, 3), (4, 7), (5, 9), (16, 16), (17, 23), (31, 8)])
def test_oracle_pyr_down_matches_opencv_steps(shape):
    rng = np.random.default_rng(shape[0] * 100 + shape[1])
    img = rng.integers(0, 256, shape).astype(np.uint8)
    H, W = shape
    sizes = {((W + 1) // 2, (H + 1) // 2)}
    for dw in range(max(1, (W - 2 + 1) // 2), (W + 2) // 2 + 1):
        for dh in range(max(1, (H - 2 + 1) // 2), (H + 2) // 2 + 1):
            if abs(2 * dw - W) <= 2 and abs(2 * dh - H) <= 2:
                sizes.add((dw, dh))
    for dw, dh in sorted(sizes):
        np.testing.assert_array_equal(oracle.pyr_down_u8(img, (dw, dh)), _pyr_down_opencv_steps(img, dw, dh))


def test_oracle_pyr_down_known_answers():
    # a constant image stays constant (weights sum to 256, +128 >> 8 exact)
    for v in (0, 1, 127, 255):
        np.testing.assert_array_equal(oracle.pyr_down_u8(np.full((9, 12), v, np.uint8)), np.full((5, 6), v))
    # a single bright pixel at (4, 4) of an 8x8 zero image: dst(2, 2) = 255*36/256 -> 36
    img = np.zeros((8, 8), np.uint8)
    img[4, 4] = 255
    d = oracle.pyr_down_u8(img)
    assert d[2, 2] == (255 * 36 + 128) >> 8
    assert d[2, 1] == (255 * 6 + 128) >> 8 and d[1, 2] == (255 * 6 + 128) >> 8
    assert d[1, 1] == (255 * 1 + 128) >> 8
    # default size rounds up; OpenCV's size assertion
    assert oracle.pyr_down_u8(np.zeros((5, 7), np.uint8)).shape == (3, 4)
    with pytest.raises(ValueError):
        oracle.pyr_down_u8(np.zeros((10, 10), np.uint8), (10, 10))  # VA:501 with rate 1
    with pytest.raises(ValueError):
        oracle.pyr_down_u8(np.zeros((10, 20), np.uint8), (5, 10))  # (H//2, W//2) read as (w, h)
