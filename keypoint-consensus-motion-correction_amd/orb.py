"""Host-side constants of the build's ORB-style detector (csrc/orb.hip).

The reference detects keypoints with OpenCV AKAZE/BRISK (VA:22-25, VA:114-116,
VA:190-192) and BASELINE config 2 names ORB; OpenCV is absent from this image, so the
detector is build-defined.  Its tables are generated here deterministically and shared
by the HIP kernels and the CPU oracle:

* the steered-BRIEF test pattern: 256 point pairs drawn once from N(0, (31/5)^2) per
  axis, rounded, restricted to the radius-13 disc (seeded numpy Generator);
* per orientation bin k (32 bins of 2 pi / 32), the pattern rotated to the bin centre
  (k + 1/2) 2 pi / 32 and rounded half-to-even: int8 [32, 512, 2] (x, y);
* the bin edges' (cos, sin) used by the exact bin tests: f64 [32, 2].
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np

N_BINS = 32
N_PAIRS = 256
PATTERN_RADIUS = 13


@dataclass(frozen=True)
class OrbParams:
    """Detector parameters (defaults follow cv2.ORB_create where they apply:
    nfeatures=500, fastThreshold=20, edgeThreshold=31 -> 16-pixel margin here,
    HARRIS_SCORE with k = 0.04; a single pyramid level)."""

    n_features: int = 500
    fast_threshold: int = 20
    harris_k: float = 0.04
    edge: int = 16


@lru_cache(maxsize=4)
def brief_pattern(seed: int = 7) -> np.ndarray:
    """[512, 2] int: points 2i and 2i+1 form BRIEF pair i."""
    rng = np.random.default_rng(seed)
    pts = []
    while len(pts) < 2 * N_PAIRS:
        x, y = np.rint(rng.normal(0.0, 31.0 / 5.0, 2))
        if x * x + y * y <= PATTERN_RADIUS * PATTERN_RADIUS:
            pts.append((int(x), int(y)))
    return np.array(pts, dtype=np.int64)


@lru_cache(maxsize=4)
def rotated_patterns(seed: int = 7) -> np.ndarray:
    p = brief_pattern(seed).astype(np.float64)
    out = np.empty((N_BINS, 2 * N_PAIRS, 2), np.int8)
    for k in range(N_BINS):
        a = (k + 0.5) * 2.0 * np.pi / N_BINS
        c, s = np.cos(a), np.sin(a)
        out[k, :, 0] = np.rint(p[:, 0] * c - p[:, 1] * s)
        out[k, :, 1] = np.rint(p[:, 0] * s + p[:, 1] * c)
    return out


@lru_cache(maxsize=1)
def bin_edges() -> np.ndarray:
    a = np.arange(N_BINS) * 2.0 * np.pi / N_BINS
    return np.ascontiguousarray(np.stack([np.cos(a), np.sin(a)], axis=1))
