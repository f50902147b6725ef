"""Host audit of the warp's fixed-pitch staged path (mode 3, warp.hip): for every tile that
warp_plan_kernel admits to mode 3, every tap that fast_rows / fastc_rows reads must lie in
the rows and columns the staging wrote, and the packed (column, row) form must not wrap.

The arithmetic is warp.hip's, restated in numpy float64 / int64 (the device code is built
with -ffp-contract=off, and rint is round-half-even on both sides):
  * invert_affine (OpenCV's in-place inversion);
  * source_box + the mode-3 admission of warp_plan_kernel (C = 1: pitch <= 144 and
    rows <= Fast<Cfg>::kRows; C = 3 / 4: pitch <= 144 and rows <= FastC<Cfg, C>::kRows);
  * the row origins of the rowtab (X0(y), Y0(y)) and lane_cols' adelta / bdelta with the
    column clamp x = min(xb + 2 lane + q, W - 1);
  * the staged area: rows [0, rows), columns [0, pitch) (fast_stage_land / fastc_stage_land
    write every (row < rows, 8-px group < pitch / 8)).
A tap (col, row) and its neighbours (col + 1, row + 1) must satisfy 0 <= col, col + 1 < pitch,
0 <= row, row + 1 < rows, and the box-relative fixed-point X (and Y) must lie in [0, 2^26)
so that the << 6 packing puts the integer part in the high half.

Usage: python tools/debug/warp_box_audit.py [--maps N] > profiles/r05_warp_box_audit.txt
"""
import argparse
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
from kcmc_amd import synthetic  # noqa: E402

TILE_W = 128
FAST_PITCH = 144
MAX_PITCH = 256
# (kTileH, kLdsElems, kRowPasses) of warp.hip's configurations
BLOCK = (56, 10240, 9)
BLOCK64 = (64, 10240, 9)
CHAN = (24, 16384, 4)


def cfg_for(C, H):
    if C == 1:
        return BLOCK64 if (H % 64 == 0 and H % 56 != 0) else BLOCK
    return CHAN


def fast_rows_limit(C, cfg):
    lds = cfg[1]
    return (lds - 8) // FAST_PITCH if C == 1 else (lds - 8) // (C * FAST_PITCH)


def invert_affine(Min):
    M = [float(v) for v in np.asarray(Min, np.float64).reshape(6)]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    return M


def rint(v):
    return np.rint(np.asarray(v, np.float64)).astype(np.int64)


def audit_map(Mfwd, H, W, C):
    """Returns (mode-3 tiles, bad taps, bad tiles, worst margins)."""
    tH, lds, passes = cfg = cfg_for(C, H)
    M = invert_affine(Mfwd)
    ntx, nty = -(-W // TILE_W), -(-H // tH)
    x = np.arange(W, dtype=np.float64)
    y = np.arange(H, dtype=np.float64)
    ad = rint(M[0] * x * 1024)             # adelta[x]
    bd = rint(M[3] * x * 1024)
    X0 = rint((M[1] * y + M[2]) * 1024) + 16
    Y0 = rint((M[4] * y + M[5]) * 1024) + 16
    n3 = bad = 0
    bad_tiles = []
    min_col_margin = min_row_margin = 1 << 30
    for ty in range(nty):
        yb = ty * tH
        yl = min(yb + tH, H) - 1
        for tx in range(ntx):
            xb = tx * TILE_W
            xl = min(xb + TILE_W, W) - 1
            a0, a1 = rint(M[0] * xb * 1024), rint(M[0] * xl * 1024)
            b0, b1 = rint(M[3] * xb * 1024), rint(M[3] * xl * 1024)
            x0 = rint((M[1] * yb + M[2]) * 1024) + 16
            x1 = rint((M[1] * yl + M[2]) * 1024) + 16
            y0 = rint((M[4] * yb + M[5]) * 1024) + 16
            y1 = rint((M[4] * yl + M[5]) * 1024) + 16
            sx0 = (min(x0, x1) + min(a0, a1)) >> 10
            sx1 = ((max(x0, x1) + max(a0, a1)) >> 10) + 1
            sy0 = (min(y0, y1) + min(b0, b1)) >> 10
            sy1 = ((max(y0, y1) + max(b0, b1)) >> 10) + 1
            lim = 30000
            small = sx0 > -lim and sx1 < lim and sy0 > -lim and sy1 < lim
            ax0 = (sx0 >> 3) << 3
            pitch = ((sx1 - ax0 + 1) + 7) & ~7
            rows = sy1 - sy0 + 1
            mode = 2
            if small and (sx1 < 0 or sx0 > W - 1 or sy1 < 0 or sy0 > H - 1):
                mode = 1
            elif small and pitch <= MAX_PITCH and rows <= 8 * passes and pitch * rows * C <= lds:
                mode = 0
            if mode == 0 and W % 8 == 0 and pitch <= FAST_PITCH and rows <= fast_rows_limit(C, cfg):
                mode = 3
            if mode != 3:
                continue
            n3 += 1
            # every row the tile's waves make (y < H) x every lane's pixel pair (clamped column)
            ys = np.arange(yb, min(yb + tH, H))
            xs = np.minimum(np.arange(xb, xb + TILE_W), W - 1)
            tX = (X0[ys][:, None] - ax0 * 1024) + ad[xs][None, :]
            tY = (Y0[ys][:, None] - sy0 * 1024) + bd[xs][None, :]
            col, row = tX >> 10, tY >> 10
            ok = (tX >= 0) & (tX < (1 << 26)) & (tY >= 0) & (tY < (1 << 26))
            ok &= (col >= 0) & (col + 1 < pitch) & (row >= 0) & (row + 1 < rows)
            nb = int((~ok).sum())
            if nb:
                bad += nb
                bad_tiles.append((tx, ty, int(ax0), int(sy0), int(pitch), int(rows)))
            min_col_margin = min(min_col_margin, int(col.min()), int(pitch - 2 - col.max()))
            min_row_margin = min(min_row_margin, int(row.min()), int(rows - 2 - row.max()))
    return n3, bad, bad_tiles, min_col_margin, min_row_margin


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", type=int, default=40, help="random maps per shape")
    args = ap.parse_args()
    # the maps of the round-4 failing run (gpurun_out/r04_k/tests.log, dbg_c4/summary.txt)
    r04 = [np.array([[1.0053911383577487, 0.0057811368368455435, 1.2748370385747876],
                     [-0.014055324654216174, 0.9906779338198224, -0.4287047332629754]]),
           np.array([[1.0078828926080385, 0.006215137383056257, -3.653160507510165],
                     [-0.006516371002192053, 0.9984373506161567, 1.0913358526368029]]),
           np.array([[1.0045123939733775, 0.0051991689442833, -0.7138911485271819],
                     [-0.0003428726917676483, 1.0085363575053359, -4.207238076060094]])]
    rng = np.random.default_rng(5)
    shapes = [(2160, 3840, 3), (2160, 3840, 4), (250, 520, 3), (240, 512, 4), (1080, 1920, 1), (512, 512, 1),
              (270, 480, 1)]
    total = {"maps": 0, "tiles3": 0, "bad": 0}
    for (H, W, C) in shapes:
        maps = [(f"r04 c4 frame {i}", m) for i, m in enumerate(r04)] if (H, W) == (2160, 3840) else []
        gt = synthetic.make_keypoints(args.maps, 8, 8, (H, W), seed=int(rng.integers(1 << 30)),
                                      model="affine").gt
        maps += [(f"c4-style gt {i}", g) for i, g in enumerate(gt)]
        # harder near-identity maps: rotations up to 4 deg, zoom 0.94..1.06, shifts to 60 px
        for i in range(args.maps):
            th = np.deg2rad(rng.uniform(-4, 4))
            s = rng.uniform(0.94, 1.06)
            A = synthetic.rigid(th, rng.uniform(-60, 60), rng.uniform(-60, 60))
            A[:, :2] *= s
            A[:, :2] += rng.uniform(-0.01, 0.01, (2, 2))
            maps.append((f"random {i}", A))
        n3 = bad = 0
        cm = rm = 1 << 30
        for name, m in maps:
            a, b, tiles, c_m, r_m = audit_map(m, H, W, C)
            n3 += a
            bad += b
            cm, rm = min(cm, c_m), min(rm, r_m)
            if b:
                print(f"  BAD {H}x{W}x{C} {name}: {b} taps outside the staged box, tiles {tiles[:8]}")
        print(f"{H}x{W}x{C}: {len(maps)} maps, {n3} mode-3 tiles, taps outside the box: {bad}, "
              f"smallest margin to the box edge: {cm} columns, {rm} rows")
        total["maps"] += len(maps)
        total["tiles3"] += n3
        total["bad"] += bad
    print(f"total: {total['maps']} maps, {total['tiles3']} mode-3 tiles audited, taps outside the staged box: "
          f"{total['bad']}")


if __name__ == "__main__":
    main()
