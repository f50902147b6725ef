"""Golden fixtures for the affine / projective RANSAC extension (BASELINE configs 3-5).

The reference fits only EuclideanTransform (VA:311); the extension runs the same
skimage call with AffineTransform (min_samples=3) and ProjectiveTransform
(min_samples=4).  Its oracle is therefore scikit-image 0.18.3 itself (the version
the reference runs against, importable in the authoring container only):

    /opt/conda/bin/python3.9 tests/golden/make_golden_models.py

Writes tests/golden/ransac_models_golden.npz (plain arrays; allow_pickle=False).
"""
import os
import warnings

import numpy as np
from skimage.measure import ransac
from skimage.transform import AffineTransform, ProjectiveTransform

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))


def apply(H, pts):
    q = np.hstack([pts, np.ones((len(pts), 1))]) @ H.T
    return q[:, :2] / q[:, 2:3]


def frames(model, rng):
    out = []
    Ns = [5, 6, 7, 8, 9, 10, 12, 16, 20, 31, 50, 64, 100, 127, 128, 129, 150, 200, 300]
    Ns += [int(n) for n in rng.integers(5, 140, 24)]
    for k, N in enumerate(Ns):
        kind = k % 6
        tpl = rng.uniform(0, 512, (N, 2))
        H = np.eye(3)
        H[:2, :2] += rng.normal(0, 0.01, (2, 2))
        H[:2, 2] = rng.normal(0, 5, 2)
        if model == "projective":
            H[2, :2] = rng.normal(0, 1e-5, 2)
        q = apply(np.linalg.inv(H), tpl)
        q += rng.normal(0, [0.3, 0.8, 1.5, 0.2, 0.5, 0.0][kind], q.shape)
        outl = rng.random(N) < [0.1, 0.3, 0.5, 0.0, 0.6, 0.2][kind]
        q[outl] = rng.uniform(0, 512, (int(outl.sum()), 2))
        if kind == 5:  # integer grid + integer shift: exact residuals, exact early exit
            tpl = np.round(tpl)
            q = tpl - np.round(H[:2, 2])
        if k % 11 == 4:  # duplicated correspondences
            q[1], tpl[1] = q[0], tpl[0]
        if k % 13 == 6:  # all frame points identical -> every hypothesis degenerate
            q[:] = q[0]
        if k % 17 == 8 and N >= 8 and model == "affine":  # collinear template points on a line
            # (not for the homography: 4 collinear points leave the DLT null space
            # 2-dimensional, so skimage's model there is whatever LAPACK returns)
            tpl[:N // 2, 1] = 100.0
        out.append((tpl.astype(np.float32).astype(np.float64), q.astype(np.float32).astype(np.float64)))
    return out


def main():
    data = {}
    for model, cls, ms in (("affine", AffineTransform, 3), ("projective", ProjectiveTransform, 4)):
        rng = np.random.default_rng({"affine": 601, "projective": 602}[model])
        fr = frames(model, rng)
        offs, tpls, qs, params, inls, nins = [0], [], [], [], [], []
        for tpl, q in fr:
            m, inl = ransac((q, tpl), cls, min_samples=ms, residual_threshold=2, max_trials=1000, random_state=42)
            params.append(np.full((3, 3), np.nan) if m is None else m.params)
            inl = np.zeros(len(q), bool) if inl is None else inl
            inls.append(inl)
            nins.append(int(inl.sum()))
            tpls.append(tpl)
            qs.append(q)
            offs.append(offs[-1] + len(q))
        data[f"{model}_kp_template"] = np.concatenate(tpls)
        data[f"{model}_kp_query"] = np.concatenate(qs)
        data[f"{model}_offsets"] = np.array(offs, np.int64)
        data[f"{model}_params"] = np.array(params)
        data[f"{model}_inliers"] = np.concatenate(inls)
        data[f"{model}_n_inliers"] = np.array(nins, np.int64)
        print(model, len(fr), "frames,", sum(np.isnan(p).any() for p in params), "without a model")
    np.savez_compressed(os.path.join(HERE, "ransac_models_golden.npz"), **data)


if __name__ == "__main__":
    main()
