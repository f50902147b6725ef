"""Seeded synthetic inputs for the hot path: jittered uint16 video and
keypoint/descriptor sets shaped like a detector's output.

No detector exists in this image (OpenCV absent), so the matcher and RANSAC are fed
synthetic keypoints: template points uniform over the frame with random uint8
descriptors; each frame sees the template points moved by that frame's ground-truth
rigid jitter plus N(0, noise) px, with 25 % of descriptor bytes perturbed by up to
+-8, 10 % of points dropped, 20 % random distractors added, and the order shuffled.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np


def rigid(theta: float, tx: float, ty: float) -> np.ndarray:
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s, tx], [s, c, ty]])


@dataclass
class KeypointSet:
    kp_tpl: np.ndarray      # [n_tpl, 2] f64 (float32-representable, like cv2 KeyPoint.pt)
    des_tpl: np.ndarray     # [n_tpl, D] u8
    kp_q: np.ndarray        # [P, 2] f64, CSR over frames
    des_q: np.ndarray       # [P, D] u8
    q_off: np.ndarray       # [F+1] i32
    gt: np.ndarray          # [F, 2, 3] frame->template rigid maps used to place the points


def ground_truth(rng: np.random.Generator, model: str, jitter: float, rot_deg: float,
                 size_hw: Tuple[int, int]) -> np.ndarray:
    """A frame -> template map: rigid jitter N(0, jitter px), N(0, rot_deg);
    "affine" adds +-1 % scale/shear; "projective" adds perspective terms ~1e-5 / px
    (scaled to the frame size) and is returned as [3, 3]."""
    A = rigid(np.deg2rad(rng.normal(0, rot_deg)), rng.normal(0, jitter), rng.normal(0, jitter))
    if model == "euclidean":
        return A
    A[:, :2] = A[:, :2] @ (np.eye(2) + rng.uniform(-0.01, 0.01, (2, 2)))
    if model == "affine":
        return A
    Hm = np.vstack([A, [0.0, 0.0, 1.0]])
    Hm[2, :2] = rng.normal(0, 1e-5 * 512.0 / max(size_hw), 2)
    return Hm


def apply_map(M: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """Apply a [2, 3] affine or [3, 3] projective map to points [n, 2]."""
    q = pts @ M[:2, :2].T + M[:2, 2]
    if M.shape == (3, 3):
        w = pts @ M[2, :2] + M[2, 2]
        q = q / w[:, None]
    return q


def make_keypoints(n_frames: int, n_tpl: int, D: int, size_hw: Tuple[int, int], seed: int = 3,
                   jitter: float = 4.0, rot_deg: float = 0.5, noise: float = 0.3, drop: float = 0.1,
                   distract: float = 0.2, perturb: int = 8, perturb_frac: float = 0.25,
                   frame_seed: Optional[int] = None, model: str = "euclidean",
                   descriptor: str = "u8", f32_noise: float = 0.05) -> KeypointSet:
    """``seed`` fixes the template; ``frame_seed`` (e.g. a rank) draws an independent
    slab of frames against that same template; ``model`` picks the ground-truth motion
    family (gt is [F, 2, 3], or [F, 3, 3] for "projective").  ``descriptor="f32"`` gives
    SIFT-style float descriptors (template N(0, 1) L2-normalised; frames add
    N(0, f32_noise) per element; distractors are fresh unit vectors)."""
    rng = np.random.default_rng(seed)
    H, W = size_hw
    kp_tpl = np.stack([rng.uniform(0, W, n_tpl), rng.uniform(0, H, n_tpl)], 1).astype(np.float32).astype(np.float64)
    if descriptor == "f32":
        des_tpl = rng.normal(0, 1, (n_tpl, D))
        des_tpl = (des_tpl / np.linalg.norm(des_tpl, axis=1, keepdims=True)).astype(np.float32)
    else:
        des_tpl = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    if frame_seed is not None:
        rng = np.random.default_rng([seed, 1 + int(frame_seed)])
    nd = int(distract * n_tpl)
    kps, dess, counts, gts = [], [], [], []
    for f in range(n_frames):
        # frame -> template map A (what RANSAC recovers); frame points = A^-1(template points)
        if model == "euclidean":
            A = rigid(np.deg2rad(rng.normal(0, rot_deg)), rng.normal(0, jitter), rng.normal(0, jitter))
        else:
            A = ground_truth(rng, model, jitter, rot_deg, size_hw)
        keep = rng.random(n_tpl) >= drop
        if model == "euclidean":  # rigid inverse (kept bit-identical to earlier rounds' fixtures)
            R, t = A[:, :2], A[:, 2]
            pts = (kp_tpl[keep] - t) @ R
        else:
            Ah = A if A.shape == (3, 3) else np.vstack([A, [0.0, 0.0, 1.0]])
            pts = apply_map(np.linalg.inv(Ah), kp_tpl[keep])
        pts = pts + rng.normal(0, noise, (int(keep.sum()), 2))
        if descriptor == "f32":
            des = (des_tpl[keep] + rng.normal(0, f32_noise, (int(keep.sum()), D))).astype(np.float32)
            extra = rng.normal(0, 1, (nd, D))
            extra = (extra / np.linalg.norm(extra, axis=1, keepdims=True)).astype(np.float32)
        else:
            des = des_tpl[keep].astype(np.int16)
            m = rng.random(des.shape) < perturb_frac
            des[m] += rng.integers(-perturb, perturb + 1, int(m.sum()), dtype=np.int16)
            des = np.clip(des, 0, 255).astype(np.uint8)
            extra = rng.integers(0, 256, (nd, D), dtype=np.uint8)
        pts = np.concatenate([pts, np.stack([rng.uniform(0, W, nd), rng.uniform(0, H, nd)], 1)])
        des = np.concatenate([des, extra])
        perm = rng.permutation(len(pts))
        kps.append(pts[perm].astype(np.float32).astype(np.float64))
        dess.append(des[perm])
        counts.append(len(pts))
        gts.append(A)
    q_off = np.zeros(n_frames + 1, np.int32)
    q_off[1:] = np.cumsum(counts)
    return KeypointSet(kp_tpl, des_tpl, np.concatenate(kps), np.concatenate(dess), q_off, np.stack(gts))


def make_texture(size_hw: Tuple[int, int], seed: int = 0, n_blobs: Optional[int] = None) -> np.ndarray:
    """Two-photon-like uint16 texture: smooth background ~2k, Gaussian blobs to ~40k,
    sparse hot pixels (so the 99.99th percentile matters, VA:481)."""
    rng = np.random.default_rng(seed)
    H, W = size_hw
    # band-limited noise: low-resolution noise upsampled by repetition + box blur
    lo = rng.normal(0, 1, (H // 8 + 2, W // 8 + 2))
    bg = np.kron(lo, np.ones((8, 8)))[:H, :W]
    k = np.ones(9) / 9.0
    bg = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, bg)
    bg = np.apply_along_axis(lambda c: np.convolve(c, k, mode="same"), 0, bg)
    img = 2000 + 300 * bg
    n_blobs = n_blobs if n_blobs is not None else max(8, H * W // 4000)
    ys, xs = rng.uniform(0, H, n_blobs), rng.uniform(0, W, n_blobs)
    sig, amp = rng.uniform(2, 5, n_blobs), rng.uniform(5000, 38000, n_blobs)
    for y, x, s, a in zip(ys, xs, sig, amp):
        y0, y1 = int(max(0, y - 4 * s)), int(min(H, y + 4 * s + 1))
        x0, x1 = int(max(0, x - 4 * s)), int(min(W, x + 4 * s + 1))
        yy, xx = np.mgrid[y0:y1, x0:x1]
        img[y0:y1, x0:x1] += a * np.exp(-((yy - y) ** 2 + (xx - x) ** 2) / (2 * s * s))
    hot = rng.random((H, W)) < 5e-5
    img[hot] = 65000
    return np.clip(img, 0, 65535).astype(np.uint16)
