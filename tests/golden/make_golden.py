"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own code.

Run in the authoring container only (the reference and scikit-image 0.18.3 are not on
the GPU box):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

What runs: /root/reference/VideoAligner.py imported as module ``VideoAligner`` with
two environment shims, both outside the reference's own logic:

* ``cv2`` is absent from this image, so a stub ``cv2`` module is injected.  Its
  detector returns keypoints/descriptors registered per frame (synthetic, seeded);
  its ``BFMatcher.knnMatch`` and ``warpAffine`` call the build's C restatements in
  ``oracle/libkcmc_oracle.so``.  Fixtures therefore pin the REFERENCE code around
  those calls (VA:196-214 filters, VA:224-286 consensus, VA:288-323 RANSAC via the
  real skimage 0.18.3, VA:325-453 affine post-processing, VA:57-158 orchestration),
  not OpenCV itself.
* The reference builds ragged ``np.array`` objects (VA:284-285), which raise on
  numpy >= 1.24.  The module's ``np`` is wrapped so that ``np.array`` of a ragged
  list returns the numpy<1.24 object array the reference was written against.

Outputs are plain arrays in .npz files (load with allow_pickle=False).
"""
import importlib.util
import os
import sys
import types
import warnings

import numpy as np

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402  (test infrastructure: the cv2 stand-in uses it)

# ----------------------------------------------------------------------------- cv2 stub
_REGISTRY = {}


class _KP:
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (float(x), float(y))


class _Detector:
    def detectAndCompute(self, image, mask):
        kp, des = _REGISTRY[np.ascontiguousarray(image).tobytes()]
        return [_KP(x, y) for x, y in kp], des


class _DMatch:
    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, q, t, d):
        self.queryIdx, self.trainIdx, self.imgIdx, self.distance = int(q), int(t), 0, float(d)


class _BFMatcher:
    def __init__(self, normType=None, crossCheck=False):
        assert normType is None and crossCheck is False

    def knnMatch(self, query, train, k=2):
        assert k == 2
        idx, dist = oracle.knn2_l2u8(query, train)
        out = []
        for i in range(idx.shape[0]):
            out.append([_DMatch(i, idx[i, k_], dist[i, k_]) for k_ in range(2) if idx[i, k_] >= 0])
        return out


def _warp_affine(image, M, dsize, flags=None):
    assert flags == 1
    return oracle.warp_affine_u16(image, M, dsize=tuple(dsize))


cv2 = types.ModuleType("cv2")
cv2.AKAZE_create = _Detector
cv2.BRISK_create = _Detector
cv2.BFMatcher = _BFMatcher
cv2.warpAffine = _warp_affine
cv2.INTER_LINEAR = 1
sys.modules["cv2"] = cv2


class _LegacyNumpy(types.ModuleType):
    """numpy with the pre-1.24 ragged np.array behaviour (object arrays)."""

    def __init__(self):
        super().__init__("numpy_legacy")
        self.__dict__.update({k: getattr(np, k) for k in dir(np) if not k.startswith("__")})

        def array(obj, *a, **kw):
            try:
                return np.array(obj, *a, **kw)
            except ValueError:
                out = np.empty(len(obj), dtype=object)
                for i, o in enumerate(obj):
                    out[i] = o
                return out

        self.array = array


spec = importlib.util.spec_from_file_location("VideoAligner", "/root/reference/VideoAligner.py")
VA_mod = importlib.util.module_from_spec(spec)
sys.modules["VideoAligner"] = VA_mod
spec.loader.exec_module(VA_mod)
VA_mod.np = _LegacyNumpy()
VideoAligner = VA_mod.VideoAligner
VideoAligner.N_JOBS_PARALLEL = 2


# ----------------------------------------------------------------------------- helpers
def csr(list_of_arrays, dtype, tail_shape=()):
    off = np.zeros(len(list_of_arrays) + 1, np.int64)
    for i, a in enumerate(list_of_arrays):
        off[i + 1] = off[i] + len(a)
    flat = np.zeros((int(off[-1]),) + tail_shape, dtype)
    for i, a in enumerate(list_of_arrays):
        if len(a):
            flat[off[i] : off[i + 1]] = np.asarray(a, dtype).reshape((-1,) + tail_shape)
    return flat, off


def rigid(theta, tx, ty):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s, tx], [s, c, ty]])


def synth_keypoints(rng, n_tpl, D, F, size, jitter=4.0, rot=0.5, noise=0.3, drop=0.1, distract=0.2,
                    perturb=8, perturb_frac=0.25):
    """Seeded template keypoints/descriptors and per-frame jittered copies."""
    kp_t = rng.uniform(0, size, (n_tpl, 2)).astype(np.float32).astype(np.float64)
    des_t = rng.integers(0, 256, (n_tpl, D), dtype=np.uint8)
    frames = []
    for f in range(F):
        A = rigid(np.deg2rad(rng.normal(0, rot)), rng.normal(0, jitter), rng.normal(0, jitter))
        keep = rng.random(n_tpl) >= drop
        pts = kp_t[keep] @ A[:, :2].T + A[:, 2] + rng.normal(0, noise, (keep.sum(), 2))
        des = des_t[keep].astype(np.int32)
        m = rng.random(des.shape) < perturb_frac
        des[m] += rng.integers(-perturb, perturb + 1, m.sum())
        des = np.clip(des, 0, 255).astype(np.uint8)
        nd = int(distract * n_tpl)
        pts = np.concatenate([pts, rng.uniform(0, size, (nd, 2))])
        des = np.concatenate([des, rng.integers(0, 256, (nd, D), dtype=np.uint8)])
        perm = rng.permutation(len(pts))
        frames.append((pts[perm].astype(np.float32).astype(np.float64), des[perm], A))
    return kp_t, des_t, frames


# ----------------------------------------------------------------------------- A. RANSAC
def make_ransac():
    from skimage.measure import ransac
    from skimage.transform import EuclideanTransform

    rng = np.random.default_rng(101)
    tpls, qs, rates, aff, inls, nin = [], [], [], [], [], []
    Ns = list(range(0, 40)) + [47, 64, 65, 96, 100, 127, 128, 129, 130, 136, 160, 200, 255, 256, 257, 300, 384, 500]
    Ns += list(rng.integers(3, 130, 60))
    for k, N in enumerate(Ns):
        N = int(N)
        kind = k % 7
        tpl = rng.uniform(0, 512, (N, 2))
        A = rigid(rng.normal(0, 0.02), rng.normal(0, 5), rng.normal(0, 5))
        q = (tpl - A[:, 2]) @ A[:, :2]  # inverse rigid of template
        q += rng.normal(0, [0.3, 0.8, 1.5, 0.2, 0.5, 1.0, 0.0][kind], q.shape)
        out = rng.random(N) < [0.1, 0.3, 0.5, 0.0, 0.7, 0.2, 0.1][kind]
        q[out] = rng.uniform(0, 512, (int(out.sum()), 2))
        if kind == 6 and N >= 3:  # integer-grid points: exact residuals, exercise ties
            tpl = np.round(tpl)
            q = np.round(tpl + np.round(A[:, 2]))
        if k % 23 == 5 and N >= 3:  # all frame points identical -> degenerate hypotheses
            q[:] = q[0]
        if k % 29 == 7 and N >= 4:  # duplicated pairs
            q[1] = q[0]
            tpl[1] = tpl[0]
        tpl = tpl.astype(np.float32).astype(np.float64)
        q = q.astype(np.float32).astype(np.float64)
        rate = 2 if k % 5 == 3 else 1
        a = VideoAligner._compute_euclidean_affine(tpl, q, rate)
        if N >= 3:
            model, inl = ransac((q, tpl), EuclideanTransform, min_samples=2, residual_threshold=2,
                                max_trials=1000, random_state=42)
            inl = np.zeros(N, bool) if inl is None else inl
        else:
            inl = np.zeros(N, bool)
        tpls.append(tpl)
        qs.append(q)
        rates.append(rate)
        aff.append(a)
        inls.append(inl)
        nin.append(int(inl.sum()))
    t_flat, off = csr(tpls, np.float64, (2,))
    q_flat, _ = csr(qs, np.float64, (2,))
    i_flat, _ = csr(inls, bool)
    np.savez_compressed(os.path.join(HERE, "ransac_golden.npz"), kp_template=t_flat, kp_query=q_flat,
                        offsets=off, spatial_rate=np.array(rates, np.int64), affine=np.array(aff),
                        inliers=i_flat, n_inliers=np.array(nin, np.int64))
    print("ransac_golden:", len(Ns), "frames")


# ----------------------------------------------------------------------------- B. matching
def make_frame_keypoints(name, seed, n_tpl, D, F, size, ties=False):
    rng = np.random.default_rng(seed)
    kp_t, des_t, frames = synth_keypoints(rng, n_tpl, D, F, size)
    if ties:  # duplicate descriptors -> equal distances, lower train index must win
        for f in range(F):
            pts, des, A = frames[f]
            des[5] = des[3]
            des[9] = des[3]
            des[11] = des_t[7]
            des[12] = des_t[7]
    out_idx, out_ord, out_kq, counts = [], [], [], []
    for f, (pts, des, A) in enumerate(frames):
        img = np.full((8, 8), f % 251, np.uint8)
        img[0, :4] = np.frombuffer(np.int32(f).tobytes(), np.uint8)
        img[1, 0] = seed % 256
        _REGISTRY[img.tobytes()] = (pts, des)
        kp_idxs, kq, log = VideoAligner._get_frame_keypoints(f, img, kp_t, des_t, "akaze")
        out_idx.append(sorted(kp_idxs))
        out_ord.append(list(kp_idxs))
        out_kq.append(kq)
        counts.append([int(line.split()[0]) for line in log.split("\n")[1:]])
    q_pts, q_off = csr([fr[0] for fr in frames], np.float64, (2,))
    q_des, _ = csr([fr[1] for fr in frames], np.uint8, (D,))
    s_flat, s_off = csr(out_idx, np.int64)
    o_flat, _ = csr(out_ord, np.int64)
    np.savez_compressed(os.path.join(HERE, name), kp_template=kp_t, des_template=des_t, kp_query=q_pts,
                        des_query=q_des, q_offsets=q_off, kp_idxs=s_flat, kp_idxs_setorder=o_flat,
                        kp_idxs_offsets=s_off, kp_query_ordered=np.array(out_kq),
                        log_counts=np.array(counts, np.int64))
    print(name, F, "frames")


# ----------------------------------------------------------------------------- C. consensus
def make_consensus():
    rng = np.random.default_rng(202)
    cases = []
    for c in range(12):
        n_tpl = int(rng.choice([40, 100, 500, 1000, 4096]))
        F = int(rng.integers(1, 40))
        p = rng.uniform(0.05, 0.9, n_tpl)
        sets = [set(np.flatnonzero(rng.random(n_tpl) < p * rng.uniform(0.3, 1.0)).tolist()) for _ in range(F)]
        if c == 3:
            sets[0] = set()
        n_kp_global = int(rng.choice([5, 10, 50, 100, 200, 500]))
        cases.append((n_tpl, sets, n_kp_global))
    va = VideoAligner()
    data = {}
    for ci, (n_tpl, sets, nk) in enumerate(cases):
        cons = va._get_consensus_kps(sets, len(sets), nk)
        va._kp_template = np.arange(n_tpl, dtype=np.float64).reshape(-1, 1) * np.array([[1.0, -1.0]])
        per_frame = []
        for s in sets:  # one frame per call: identical order, no ragged array
            tk, qk = va._lookup_consensus_kps(cons, [s], [np.zeros((n_tpl, 2))])
            per_frame.append(np.asarray(tk[0])[:, 0].astype(np.int64) if len(tk[0]) else np.zeros(0, np.int64))
        f_flat, f_off = csr([sorted(s) for s in sets], np.int64)
        l_flat, l_off = csr(per_frame, np.int64)
        data[f"c{ci}_n_tpl"] = np.int64(n_tpl)
        data[f"c{ci}_n_kp_global"] = np.int64(nk)
        data[f"c{ci}_frames"] = f_flat
        data[f"c{ci}_frames_off"] = f_off
        data[f"c{ci}_consensus_setorder"] = np.array(list(cons), np.int64)
        data[f"c{ci}_lookup"] = l_flat
        data[f"c{ci}_lookup_off"] = l_off
    data["n_cases"] = np.int64(len(cases))
    # too few keypoints -> AlignmentError
    try:
        va._get_consensus_kps([{1, 2}, {2, 3}], 2, 10)
        data["too_few_raises"] = np.int64(0)
    except VideoAligner.AlignmentError:
        data["too_few_raises"] = np.int64(1)
    np.savez_compressed(os.path.join(HERE, "consensus_golden.npz"), **data)
    print("consensus_golden:", len(cases), "cases")


# ----------------------------------------------------------------------------- D. affines
def make_affines():
    rng = np.random.default_rng(303)
    data = {}
    patterns = {
        "none": [],
        "lead": [0, 1, 2],
        "trail": [17, 18, 19],
        "mid": [4, 5, 9],
        "mixed": [0, 3, 4, 10, 11, 12, 19],
        "all_but_one": [i for i in range(20) if i != 7],
    }
    for name, miss in patterns.items():
        aff = np.stack([rigid(rng.normal(0, 0.01), rng.normal(0, 3), rng.normal(0, 3)) for _ in range(20)])
        for i in miss:
            aff[i] = np.nan
        samp = [a for a in aff]
        for rate in (1, 3):
            expanded, skipped = VideoAligner._process_affines(samp, rate)
            interp, interp_idx = VideoAligner._interpolate_affines(expanded.copy())
            eu = VideoAligner._get_euclidean_transforms(interp)
            data[f"{name}_r{rate}_in"] = aff
            data[f"{name}_r{rate}_expanded"] = expanded
            data[f"{name}_r{rate}_skipped"] = np.array(skipped, np.int64)
            data[f"{name}_r{rate}_interp"] = interp
            data[f"{name}_r{rate}_interp_idx"] = np.array(interp_idx, np.int64)
            data[f"{name}_r{rate}_euclid"] = eu
    try:
        VideoAligner._interpolate_affines(np.full((4, 2, 3), np.nan))
        data["all_nan_raises"] = np.int64(0)
    except VideoAligner.AlignmentError:
        data["all_nan_raises"] = np.int64(1)
    np.savez_compressed(os.path.join(HERE, "affines_golden.npz"), **data)
    print("affines_golden")


# ----------------------------------------------------------------------------- E. pipeline
def make_pipeline():
    rng = np.random.default_rng(404)
    F, H, W = 14, 48, 64
    imgs = (rng.integers(1500, 2500, (F, H, W))).astype(np.uint16)
    yy, xx = np.mgrid[0:H, 0:W]
    for _ in range(12):
        cy, cx, s = rng.uniform(0, H), rng.uniform(0, W), rng.uniform(2, 5)
        imgs += (30000 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))).astype(np.uint16)
    imgs[3, 5, 7] = 65000  # hot pixel
    va = VideoAligner()
    brightest = va._get_brightest_px(imgs)
    template_idx = int(F * va.TEMPLATE_FRAME_LOC)
    imgs8, tmpl8 = va._max_scale_images(imgs, imgs[template_idx], brightest, np.uint8)
    kp_t, des_t, frames = synth_keypoints(rng, 60, 61, F, 64, jitter=2.0, rot=0.3)
    _REGISTRY[np.ascontiguousarray(tmpl8).tobytes()] = (kp_t, des_t)
    # frames 2 and 9 get nearly nothing matched -> NaN -> interpolated
    for f in range(F):
        pts, des, A = frames[f]
        if f in (2, 9):
            des = rng.integers(0, 256, des.shape, dtype=np.uint8)
        if f == template_idx:
            continue
        _REGISTRY[np.ascontiguousarray(imgs8[f]).tobytes()] = (pts, des)
    # the template frame is also a sample frame: it matches itself exactly
    _REGISTRY[np.ascontiguousarray(imgs8[template_idx]).tobytes()] = (kp_t, des_t)
    aligned, eu, skipped = va.align_images(imgs, n_kp_global=25, detector_algorithm="akaze", frame_rate=30)
    q_pts, q_off = csr([fr[0] if f != template_idx else kp_t for f, fr in enumerate(frames)], np.float64, (2,))
    q_des, _ = csr(
        [_REGISTRY[np.ascontiguousarray(imgs8[f]).tobytes()][1] for f in range(F)], np.uint8, (61,))
    np.savez_compressed(os.path.join(HERE, "pipeline_golden.npz"), images=imgs, kp_template=kp_t,
                        des_template=des_t, kp_query=q_pts, des_query=q_des, q_offsets=q_off,
                        aligned=aligned, euclidean=eu, skipped=np.array(skipped, np.int64),
                        interpolated=np.array(va.interpolated_idxs, np.int64), brightest=np.float64(brightest),
                        n_kp_global=np.int64(25))
    print("pipeline_golden: skipped", skipped, "interpolated", va.interpolated_idxs)


# ----------------------------------------------------------------------------- F. preprocessing
def make_preprocess():
    rng = np.random.default_rng(505)
    data = {}
    for k, shape in enumerate([(3, 17, 19), (7, 64, 48), (2, 5, 5)]):
        imgs = rng.integers(0, 65536, shape).astype(np.uint16)
        if k == 1:
            imgs = (imgs // 16).astype(np.uint16)
        b = VideoAligner._get_brightest_px(imgs)
        i8, t8 = VideoAligner._max_scale_images(imgs, imgs[len(imgs) // 2], b, np.uint8)
        data[f"p{k}_images"] = imgs
        data[f"p{k}_brightest"] = np.float64(b)
        data[f"p{k}_u8"] = i8
        data[f"p{k}_tpl_u8"] = t8
    data["n_cases"] = np.int64(3)
    np.savez_compressed(os.path.join(HERE, "preprocess_golden.npz"), **data)
    print("preprocess_golden")


if __name__ == "__main__":
    make_ransac()
    make_frame_keypoints("match_golden_akaze.npz", 11, 200, 61, 24, 512)
    make_frame_keypoints("match_golden_orb.npz", 12, 150, 32, 16, 1080, ties=True)
    make_consensus()
    make_affines()
    make_pipeline()
    make_preprocess()
