"""Worker processes of bench.py's cpu_baseline leg -- TEST/BASELINE INFRASTRUCTURE ONLY.

The reference runs its per-frame stages in a joblib process pool with one process per
core (VideoAligner._parallelize, VA:460-465); the CPU baseline mirrors that: the oracle
restatement of each per-frame stage (C knnMatch + the reference's numpy filters, the
numpy/LAPACK restatement of skimage 0.18.3 ransac, C warpAffine/warpPerspective) runs
in worker processes over contiguous frame chunks, the consensus (VA:224-286) in the
parent, as in the reference.  Never imported by the product path.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

_S = {}


ARRAYS = ("des_tpl", "kp_tpl", "des_q", "kp_q", "q_off", "base")


def init(data, model, descriptor):
    """``data``: the arrays themselves (a single in-process worker) or the directory they
    were saved to as .npy files (pool workers memory-map them: with one process per core
    of a large host, pickling ~50 MB of keypoints into every worker would dominate)."""
    from threadpoolctl import threadpool_limits

    threadpool_limits(1)  # one single-threaded process per core, like the reference's pool
    import oracle

    if isinstance(data, str):
        data = {k: np.load(os.path.join(data, k + ".npy"), mmap_mode="r") for k in ARRAYS}
    _S.update(data, model=model, descriptor=descriptor, oracle=oracle)


def ping(_):
    return os.getpid()


def match_chunk(frames):
    """_get_frame_keypoints' matching half (VA:194-214) per frame: (survivor set, kq)."""
    o, S = _S["oracle"], _S
    knn = o.knn2_l2f32 if S["descriptor"] == "f32" else o.knn2_l2u8
    out = []
    for f in frames:
        a, b = S["q_off"][f], S["q_off"][f + 1]
        idx, dist = knn(S["des_tpl"], S["des_q"][a:b])
        s, kq, _ = o.filter_matches(idx, dist, S["kp_tpl"], S["kp_q"][a:b])
        out.append((s, kq))
    return out


def ransac_warp_chunk(items):
    """_compute_euclidean_affine (VA:288-323) + _apply_affine (VA:455-458) per frame."""
    o, S = _S["oracle"], _S
    model = S["model"]
    skip = {"euclidean": 3, "affine": 4, "projective": 5}[model]
    for kq, L in items:
        L = np.asarray(L, np.int64)
        if len(L) < skip:
            p = np.full((3, 3) if model == "projective" else (2, 3), np.nan)
        elif model == "euclidean":
            p, _ = o.ransac_rigid_skimage(kq[L], S["kp_tpl"][L])
        else:
            p, _ = o.ransac_model_skimage(kq[L], S["kp_tpl"][L], model)
            p = p[:2] if model == "affine" else p
        if model == "projective":
            o.warp_perspective_u16(S["base"], p)
        else:
            o.warp_affine_u16(S["base"], p)
    return len(items)
