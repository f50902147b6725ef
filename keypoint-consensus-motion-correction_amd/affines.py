"""Host-side affine post-processing between RANSAC and the warp (VA:325-453).

O(F) scalar work on a few KB; it stays on the host, as in the reference, but is
written with array operations and only loops over NaN gaps.  Results are
identical to the reference's (pinned by tests/golden/affines_golden.npz), including
its quirks: trailing extrapolated frames are not reported as interpolated
(VA:400), rotation is recovered as arccos(a00) (sign lost, VA:452), and gap
interpolation lerps arccos/arcsin of the four rotation entries independently
(VA:423-436).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


class AlignmentError(BaseException):
    """Raised when alignment cannot proceed (VA:16-17); same base class as the reference."""


def _nan_rows(a: np.ndarray) -> np.ndarray:
    """Rows of [n, ...] holding any NaN.  One vectorised pass per matrix entry: numpy's
    any(axis=1) over a short trailing axis costs ~25 ns per row, 0.4 ms per call at the
    16 000 frames every rank post-processes in an 8-GPU job."""
    flat = a.reshape(len(a), -1)
    m = np.isnan(flat[:, 0]) if flat.shape[1] else np.zeros(len(a), bool)
    for j in range(1, flat.shape[1]):
        m |= np.isnan(flat[:, j])
    return m


def process_affines(affines_sample: Sequence[np.ndarray], frame_downsample_rate: int) -> Tuple[np.ndarray, List[int]]:
    """VA:326-345: stack, record NaN sample frames, NaN-pad the temporally skipped frames."""
    a = affines_sample if isinstance(affines_sample, np.ndarray) else np.stack(affines_sample)
    rate = int(frame_downsample_rate)
    skipped = [int(i) * rate for i in np.flatnonzero(_nan_rows(a))]
    dtype = np.result_type(a.dtype, np.float64)
    if rate == 1:
        out = np.array(a, dtype=dtype, copy=True)
    else:
        out = np.full((len(a) * rate,) + a.shape[1:], np.nan, dtype=dtype)
        out[::rate] = a
    return out, skipped


def _lerp_gap(a_prev: np.ndarray, a_next: np.ndarray, x_lo: int, x_hi: int, xs: np.ndarray) -> np.ndarray:
    """VA:410-437 for one gap: scipy interp1d(kind='linear') evaluated the way scipy does,
    y = slope * (x - x_lo) + y_lo with slope = (y_hi - y_lo) / (x_hi - x_lo)."""
    base = np.array((a_prev, a_next), dtype=np.float64)
    base[:, 0, 0] = np.arccos(base[:, 0, 0])
    base[:, 0, 1] = np.arcsin(base[:, 0, 1])
    base[:, 1, 0] = np.arcsin(base[:, 1, 0])
    base[:, 1, 1] = np.arccos(base[:, 1, 1])
    y_lo, y_hi = base[0], base[1]
    slope = (y_hi - y_lo) / (float(x_hi) - float(x_lo))
    out = slope[None] * (xs.astype(np.float64) - float(x_lo))[:, None, None] + y_lo[None]
    out[:, 0, 0] = np.cos(out[:, 0, 0])
    out[:, 0, 1] = np.sin(out[:, 0, 1])
    out[:, 1, 0] = np.sin(out[:, 1, 0])
    out[:, 1, 1] = np.cos(out[:, 1, 1])
    return out


def interpolate_affines(affines: np.ndarray) -> Tuple[np.ndarray, List[int]]:
    """VA:347-407: fill NaN frames (edge-fill at the ends, per-gap lerp inside)."""
    aff = np.array(affines, dtype=np.float64, copy=True)
    n = len(aff)
    missing = _nan_rows(aff)
    if not missing.any():
        return aff, []
    if missing.all():
        raise AlignmentError(
            "No transformations were calculated because too few keypoints were identified "
            "(probably because too few keypoints were identified)"
        )
    present = np.flatnonzero(~missing)
    interpolated: List[int] = []
    first = int(present[0])
    if first > 0:  # extrapolate leading frames (VA:383-387)
        aff[:first] = aff[first]
        interpolated += list(range(first))
    gaps = np.flatnonzero(np.diff(present) > 1)
    for g in gaps:  # interior gaps (VA:389-395)
        lo, hi = int(present[g]), int(present[g + 1])
        xs = np.arange(lo + 1, hi)
        aff[lo + 1 : hi] = _lerp_gap(aff[lo], aff[hi], lo, hi, xs)
        interpolated += list(range(lo + 1, hi))
    last = int(present[-1])
    if last < n - 1:  # extrapolate trailing frames (VA:397-400: reported range is empty)
        aff[last + 1 :] = aff[last]
    if aff.shape[1:] != (2, 3):
        raise AlignmentError(
            "An error occurred interpolating affine transforms for frames which had no affine transform estimate"
        )
    return aff, interpolated


def interpolate_linear(maps: np.ndarray) -> Tuple[np.ndarray, List[int]]:
    """Gap filling for the extension models (affine [n, 2, 3], projective [n, 3, 3]):
    the reference's edge-fill and reporting rules (VA:347-407) with entry-wise linear
    interpolation inside gaps (its arccos/arcsin lerp, VA:423-436, assumes rotation
    entries and returns NaN for scaled matrices)."""
    m = np.array(maps, dtype=np.float64, copy=True)
    n = len(m)
    missing = _nan_rows(m)
    if not missing.any():
        return m, []
    if missing.all():
        raise AlignmentError(
            "No transformations were calculated because too few keypoints were identified "
            "(probably because too few keypoints were identified)"
        )
    present = np.flatnonzero(~missing)
    interpolated: List[int] = []
    first = int(present[0])
    if first > 0:
        m[:first] = m[first]
        interpolated += list(range(first))
    for g in np.flatnonzero(np.diff(present) > 1):
        lo, hi = int(present[g]), int(present[g + 1])
        t = (np.arange(lo + 1, hi, dtype=np.float64) - lo) / float(hi - lo)
        m[lo + 1 : hi] = m[lo][None] + (m[hi] - m[lo])[None] * t[:, None, None]
        interpolated += list(range(lo + 1, hi))
    last = int(present[-1])
    if last < n - 1:
        m[last + 1 :] = m[last]
    return m, interpolated


def _fill_span(m: np.ndarray, xs: np.ndarray, lerp: bool) -> Tuple[np.ndarray, List[int]]:
    """The gap filling of interpolate_affines (lerp=True, VA:347-407) / interpolate_linear
    over rows m whose global frame indices are xs (consecutive, at least one row without
    NaN): leading rows take the first model (reported), interior gaps are interpolated
    between their two neighbours at their global indices (reported), trailing rows take the
    last model (not reported, VA:400).  Returns (filled rows, reported global indices)."""
    missing = _nan_rows(m)
    present = np.flatnonzero(~missing)
    reported: List[int] = []
    first = int(present[0])
    if first > 0:
        m[:first] = m[first]
        reported += xs[:first].tolist()
    for g in np.flatnonzero(np.diff(present) > 1):
        lo, hi = int(present[g]), int(present[g + 1])
        x_lo, x_hi = int(xs[lo]), int(xs[hi])
        gx = xs[lo + 1 : hi]
        if lerp:
            m[lo + 1 : hi] = _lerp_gap(m[lo], m[hi], x_lo, x_hi, gx)
        else:
            t = (gx.astype(np.float64) - x_lo) / float(x_hi - x_lo)
            m[lo + 1 : hi] = m[lo][None] + (m[hi] - m[lo])[None] * t[:, None, None]
        reported += gx.tolist()
    last = int(present[-1])
    if last < len(m) - 1:
        m[last + 1 :] = m[last]
    return m, reported


def fill_gaps_slab(params: np.ndarray, f0: int, prev: Optional[Tuple[int, np.ndarray]],
                   nxt: Optional[Tuple[int, np.ndarray]], lerp: bool) -> Tuple[np.ndarray, List[int], List[int]]:
    """NaN-gap filling of one rank's frames [f0, f0 + n) of a frame-sharded job (frame
    downsample rate 1), equal to the rows [f0, f0 + n) of interpolate_affines /
    interpolate_linear over all frames: ``prev`` = (global index, model) of the last frame
    with a model before f0 on any rank, ``nxt`` the first one after the slab (None: there
    is none).  Only those two neighbours cross ranks, so a rank's work is O(its frames).
    Returns (filled [n, ...], skipped global indices (VA:339), reported interpolated
    global indices of this slab).  AlignmentError when no frame of the job has a model."""
    m = np.array(params, dtype=np.float64, copy=True)
    n = len(m)
    skipped = (np.flatnonzero(_nan_rows(m)) + f0).tolist() if n else []
    if not skipped:
        return m, [], []
    rows, xs, lo = [m], [np.arange(f0, f0 + n)], 0
    if prev is not None:
        rows.insert(0, np.asarray(prev[1], dtype=np.float64).reshape((1,) + m.shape[1:]))
        xs.insert(0, np.array([prev[0]]))
        lo = 1
    if nxt is not None:
        rows.append(np.asarray(nxt[1], dtype=np.float64).reshape((1,) + m.shape[1:]))
        xs.append(np.array([nxt[0]]))
    ext, gx = np.concatenate(rows), np.concatenate(xs)
    if _nan_rows(ext).all():
        raise AlignmentError(
            "No transformations were calculated because too few keypoints were identified "
            "(probably because too few keypoints were identified)"
        )
    ext, reported = _fill_span(ext, gx, lerp)
    lo_x, hi_x = f0, f0 + n
    return ext[lo : lo + n], skipped, [x for x in reported if lo_x <= x < hi_x]


def euclidean_transforms(affines: np.ndarray) -> np.ndarray:
    """VA:440-453: [x_translation, y_translation, arccos(a00)] per frame."""
    t = np.zeros((affines.shape[0], 3))
    t[:, :2] = affines[:, :2, 2]
    with np.errstate(invalid="ignore"):  # arccos(a00 > 1) -> NaN, as in the reference
        t[:, 2] = np.arccos(affines[:, 0, 0])
    return t
