"""Host-side parts of the product that run without a GPU: the native hypothesis-table
generator, the native CPython-set consensus, the affine post-processing and the
VideoAligner host helpers -- each against the oracle and the reference goldens."""
import numpy as np
import pytest

import oracle
from conftest import load_golden
from kcmc_amd import VideoAligner, affines, stages


# ------------------------------------------------------------ hypothesis tables
@pytest.mark.parametrize("n", list(range(3, 40)) + [64, 100, 127, 128, 129, 255, 500, 1000, 4096])
def test_native_hypothesis_table_matches_numpy(n):
    assert np.array_equal(stages.hypothesis_table(n, 1000, 42), oracle.hypothesis_table(n, 1000, 42))


def test_native_hypothesis_table_other_seeds_and_sizes():
    for seed in (0, 1, 2**32 - 1):
        rs = np.random.RandomState(seed)
        exp = np.array([rs.choice(50, 3, replace=False) for _ in range(20)])
        assert np.array_equal(stages.hypothesis_table(50, 20, seed, 3), exp)


# ------------------------------------------------------------ consensus
def _bits(sets, n_tpl):
    words = (n_tpl + 31) // 32
    kb = np.zeros((len(sets), words), np.uint32)
    for f, s in enumerate(sets):
        for i in s:
            kb[f, i >> 5] |= np.uint32(1 << (i & 31))
    return kb


def _check_consensus(sets, n_tpl, n_kp_global, n_min=5):
    try:
        cons_set, order, votes = oracle.consensus(sets, n_kp_global, n_min)
    except RuntimeError:
        with pytest.raises(VideoAligner.AlignmentError):
            stages.consensus(_bits(sets, n_tpl), n_tpl, n_kp_global, n_min)
        return
    c = stages.consensus(_bits(sets, n_tpl), n_tpl, n_kp_global, n_min)
    assert c.order.tolist() == list(order)
    assert c.votes.tolist() == list(votes)
    lists = oracle.lookup(cons_set, sets)
    for f, L in enumerate(lists):
        assert c.pt_idx[c.pt_off[f]:c.pt_off[f + 1]].tolist() == L


def test_native_consensus_matches_cpython_random():
    rng = np.random.default_rng(7)
    for case in range(60):
        n_tpl = int(rng.choice([8, 33, 100, 500, 1000, 4096, 9000]))
        F = int(rng.integers(1, 50))
        p = rng.uniform(0.0, 0.9, n_tpl) * rng.uniform(0.1, 1.0)
        # sets built from ascending lists, exactly like VA:214
        sets = [set(np.flatnonzero(rng.random(n_tpl) < p).tolist()) for _ in range(F)]
        n_kp_global = int(rng.choice([1, 5, 10, 50, 100, 200, 500, 5000]))
        _check_consensus(sets, n_tpl, n_kp_global)


def test_native_consensus_many_ties():
    # all counts equal -> most_common order is first-occurrence (set iteration) order
    sets = [set(range(0, 300, 3)), set(range(0, 300, 3))]
    _check_consensus(sets, 300, 17)
    _check_consensus([set(range(1000))], 1000, 1000)
    _check_consensus([set([999, 64, 65, 3, 1029 % 1000])], 1000, 5)


def test_native_consensus_sorted_order_shortcut_boundaries():
    # per-frame results whose final set table is / is not larger than their largest key
    # (the native code lists the former in ascending order and replays the latter):
    # intersection sizes around the 128 -> 512 table growth (76 / 77 elements), small
    # sets of small keys, and sets with keys just above / below the table size
    rng = np.random.default_rng(3)
    n_tpl = 600
    common = list(range(0, 600, 4))  # 150 keys seen in every frame -> the consensus
    sets = [set(common)]
    for m in (1, 2, 5, 19, 20, 76, 77, 78, 120, 150):
        # built from ascending lists, like VA:214
        sets.append(set(sorted(rng.choice(common, m, replace=False).tolist())))
    sets += [set([0, 4, 8]), set([4, 28]), set([0, 32]), set([124, 128]), set([508, 512, 516])]
    sets += [set(common[:76]), set(common[-76:]), set(common[:77]), set(common[-77:])]
    _check_consensus(sets, n_tpl, 150)
    _check_consensus(sets, n_tpl, 40)


def test_native_consensus_many_frames_threaded_vote():
    """>= 8192 frames (the all-gathered bitmasks of a multi-GPU job): the vote counts are
    split over threads; counts, first-occurrence order and point lists equal CPython's.
    Key 0 only in the last frame and the top keys with counts that differ by one make
    the per-thread partial sums and the any-mask merge observable."""
    rng = np.random.default_rng(5)
    n_tpl, F = 300, 9000
    p = rng.uniform(0.05, 0.6, n_tpl)
    p[0] = 0.0
    sets = [set(np.flatnonzero(rng.random(n_tpl) < p).tolist()) for _ in range(F)]
    sets[-1] = set(sorted(sets[-1] | {0}))  # built from an ascending list, like VA:214
    _check_consensus(sets, n_tpl, 60)
    _check_consensus(sets, n_tpl, n_tpl)


def test_native_consensus_frame_slices_match_full():
    """kcmc_consensus_slice: the consensus of every frame, the point lists of a frame
    range (a rank's share of a sharded job) == the full result's lists for those frames."""
    rng = np.random.default_rng(11)
    n_tpl, F = 500, 90
    sets = [set(np.flatnonzero(rng.random(n_tpl) < 0.7).tolist()) for _ in range(F)]
    kb = _bits(sets, n_tpl)
    full = stages.consensus(kb, n_tpl, 100, 1)
    for f0, f1 in [(0, F), (0, 1), (13, 57), (57, 90), (89, 90), (40, 40)]:
        part = stages.consensus(kb, n_tpl, 100, 1, frames=(f0, f1))
        assert np.array_equal(part.order, full.order) and np.array_equal(part.votes, full.votes)
        lo, hi = full.pt_off[f0], full.pt_off[f1]
        assert np.array_equal(part.pt_off, full.pt_off[f0:f1 + 1] - lo)
        assert np.array_equal(part.pt_idx, full.pt_idx[lo:hi])
    with pytest.raises(ValueError):
        stages.consensus(kb, n_tpl, 100, 1, frames=(5, 91))


def test_native_consensus_too_few_raises():
    with pytest.raises(VideoAligner.AlignmentError):
        stages.consensus(_bits([{1, 2}, {2, 3}], 10), 10, 10, 5)


def test_native_consensus_vs_reference_golden():
    g = load_golden("consensus_golden.npz")
    for c in range(int(g["n_cases"])):
        n_tpl = int(g[f"c{c}_n_tpl"])
        fo, fl = g[f"c{c}_frames_off"], g[f"c{c}_frames"]
        sets = [set(fl[fo[i]:fo[i + 1]].tolist()) for i in range(len(fo) - 1)]
        res = stages.consensus(_bits(sets, n_tpl), n_tpl, int(g[f"c{c}_n_kp_global"]), 5)
        assert sorted(res.order.tolist()) == sorted(g[f"c{c}_consensus_setorder"].tolist())
        lo, ll = g[f"c{c}_lookup_off"], g[f"c{c}_lookup"]
        assert np.array_equal(res.pt_off, lo)
        assert np.array_equal(res.pt_idx, ll)


# ------------------------------------------------------------ affine post-processing
def test_affines_vs_reference_golden():
    g = load_golden("affines_golden.npz")
    names = sorted({k.rsplit("_r", 1)[0] for k in g.files if k.endswith("_in")})
    for name in names:
        for rate in (1, 3):
            p = f"{name}_r{rate}"
            exp, skipped = affines.process_affines(list(g[p + "_in"]), rate)
            np.testing.assert_array_equal(exp, g[p + "_expanded"])
            assert skipped == g[p + "_skipped"].tolist()
            itp, idx = affines.interpolate_affines(exp)
            # arccos/arcsin/cos/sin differ by ~1 ulp between numpy builds (the golden was
            # made with numpy 1.26); everything else is exact
            np.testing.assert_allclose(itp, g[p + "_interp"], rtol=1e-13, atol=1e-15)
            assert idx == g[p + "_interp_idx"].tolist()
            np.testing.assert_allclose(affines.euclidean_transforms(itp), g[p + "_euclid"], rtol=1e-13, atol=1e-15)
    with pytest.raises(VideoAligner.AlignmentError):
        affines.interpolate_affines(np.full((4, 2, 3), np.nan))


def test_gap_lerp_matches_scipy_interp1d():
    from scipy.interpolate import interp1d

    rng = np.random.default_rng(9)
    for _ in range(50):
        lo = int(rng.integers(0, 20))
        hi = lo + int(rng.integers(2, 9))
        base = np.stack([np.array([[np.cos(t), -np.sin(t), rng.normal()], [np.sin(t), np.cos(t), rng.normal()]])
                         for t in rng.normal(0, 0.05, 2)])
        b = base.copy()
        b[:, 0, 0] = np.arccos(b[:, 0, 0])
        b[:, 0, 1] = np.arcsin(b[:, 0, 1])
        b[:, 1, 0] = np.arcsin(b[:, 1, 0])
        b[:, 1, 1] = np.arccos(b[:, 1, 1])
        it = interp1d([lo, hi], b, axis=0)
        xs = np.arange(lo + 1, hi)
        got = affines._lerp_gap(base[0], base[1], lo, hi, xs)
        for k, j in enumerate(xs):
            a = it(j)
            a[0, 0], a[0, 1], a[1, 0], a[1, 1] = np.cos(a[0, 0]), np.sin(a[0, 1]), np.sin(a[1, 0]), np.cos(a[1, 1])
            np.testing.assert_array_equal(got[k], a)


# ------------------------------------------------------------ VideoAligner host helpers
def test_preprocessing_vs_reference_golden():
    g = load_golden("preprocess_golden.npz")
    for k in range(int(g["n_cases"])):
        imgs = g[f"p{k}_images"]
        b = VideoAligner._get_brightest_px(imgs)
        assert b == g[f"p{k}_brightest"]
        i8, t8 = VideoAligner._max_scale_images(imgs, imgs[len(imgs) // 2], b, np.uint8)
        np.testing.assert_array_equal(i8, g[f"p{k}_u8"])
        np.testing.assert_array_equal(t8, g[f"p{k}_tpl_u8"])


def test_consensus_helpers_vs_reference_golden():
    g = load_golden("consensus_golden.npz")
    va = VideoAligner()
    for c in range(int(g["n_cases"])):
        n_tpl = int(g[f"c{c}_n_tpl"])
        fo, fl = g[f"c{c}_frames_off"], g[f"c{c}_frames"]
        sets = [set(fl[fo[i]:fo[i + 1]].tolist()) for i in range(len(fo) - 1)]
        cons = va._get_consensus_kps(sets, len(sets), int(g[f"c{c}_n_kp_global"]))
        assert list(cons) == g[f"c{c}_consensus_setorder"].tolist()
        va._kp_template = np.arange(n_tpl, dtype=np.float64).reshape(-1, 1) * np.array([[1.0, -1.0]])
        tk, _ = va._lookup_consensus_kps(cons, sets, [np.zeros((n_tpl, 2))] * len(sets))
        lo, ll = g[f"c{c}_lookup_off"], g[f"c{c}_lookup"]
        for i in range(len(sets)):
            got = np.asarray(tk[i]).reshape(-1, 2)[:, 0].astype(np.int64).tolist()
            assert got == ll[lo[i]:lo[i + 1]].tolist()
    with pytest.raises(VideoAligner.AlignmentError):
        va._get_consensus_kps([{1, 2}, {2, 3}], 2, 10)


def test_api_surface_matches_reference():
    import kcmc_amd

    for name in ("FRAME_SAMPLE_RATE", "SPATIAL_DOWNSAMPLE_RATE", "N_JOBS_PARALLEL", "DETECTOR_CONSTRUCTOR_DICT",
                 "N_KP_GLOBAL_MIN", "N_KP_FRAME_SKIP", "TEMPLATE_FRAME_LOC", "MAX_FRAC_INTERPOLATED",
                 "DESCRIPTOR_DISTANCE_RATIO_THRESH", "MEDIAN_KEYPOINT_INLIER_DISTANCE_RANGE",
                 "IMAGE_NORM_MAX_PERCENTILE", "MAX_PIXEL_UINT8", "RANSAC_MIN_SAMPLES", "RANSAC_RESIDUAL_THRESH",
                 "RANSAC_MAX_TRIALS", "RANDOM_SEED", "align_images", "_get_frame_keypoints", "_get_consensus_kps",
                 "_lookup_consensus_kps", "_compute_euclidean_affine", "_process_affines", "_interpolate_affines",
                 "_interpolate_affines_frame_range", "_get_euclidean_transforms", "_apply_affine", "_parallelize",
                 "_parallelize_i", "_convert_to_array", "_get_brightest_px", "_max_scale_images", "_downsample"):
        assert hasattr(VideoAligner, name), name
    assert {"akaze", "brisk"} <= set(VideoAligner.DETECTOR_CONSTRUCTOR_DICT)  # the reference's (VA:22-25); "orb" is the GPU extension
    assert issubclass(VideoAligner.AlignmentError, BaseException)
    assert kcmc_amd.LoResVideoAligner.SPATIAL_DOWNSAMPLE_RATE == 2
    assert (VideoAligner.RANSAC_MAX_TRIALS, VideoAligner.RANDOM_SEED, VideoAligner.N_KP_FRAME_SKIP) == (1000, 42, 3)


def test_percentile_restatement_matches_numpy():
    """stages._numpy_linear_percentile (the host half of the device percentile, VA:481)
    equals np.percentile exactly, for the reference's 99.99 and other quantiles."""
    from kcmc_amd.stages import _numpy_linear_percentile

    rng = np.random.default_rng(0)
    for _ in range(2000):
        n = int(rng.integers(1, 4000))
        a = rng.integers(0, int(rng.choice([2, 10, 300, 65536])), n).astype(np.uint16)
        q = float(rng.choice([99.99, 50.0, 0.0, 100.0, 12.5, rng.uniform(0, 100)]))
        s = np.sort(a)
        assert _numpy_linear_percentile(n, q, lambda r: int(s[r])) == np.percentile(a, q)


def test_max_scale_lut_matches_reference_expression():
    from kcmc_amd.stages import max_scale_lut

    g = load_golden("preprocess_golden.npz")
    for k in range(int(g["n_cases"])):
        imgs, b = g[f"p{k}_images"], float(g[f"p{k}_brightest"])
        assert np.array_equal(max_scale_lut(b)[imgs], g[f"p{k}_u8"])


# ------------------------------------------------------------ consensus in three parts
def _split_consensus(kb, n_tpl, n_kp_global, n_min, cuts):
    """vote per frame range ("rank"), merge, lookup per range: the sharded consensus."""
    votes = np.stack([stages.consensus_vote_host(kb[a:b], n_tpl, a) for a, b in zip(cuts, cuts[1:])])
    rng = np.random.default_rng(len(cuts))
    choice = stages.consensus_merge(votes[rng.permutation(len(votes))], n_tpl, n_kp_global, n_min)
    offs, idxs = [0], []
    for a, b in zip(cuts, cuts[1:]):
        po, pi = stages.consensus_lookup_host(kb[a:b], n_tpl, choice.cons_iter)
        offs.extend((offs[-1] + po[1:]).tolist())
        idxs.append(pi)
    return choice, np.asarray(offs, np.int32), np.concatenate(idxs) if idxs else np.zeros(0, np.int32)


def test_three_part_consensus_equals_cpython_and_full():
    """vote (per frame range) -> merge (ranks in any order) -> lookup (per frame range) gives
    CPython's Counter.most_common order, counts and every frame's set-order point list --
    the same as the one-shot native consensus."""
    rng = np.random.default_rng(21)
    for case in range(40):
        n_tpl = int(rng.choice([8, 33, 100, 500, 1000, 4096]))
        F = int(rng.integers(1, 40))
        p = rng.uniform(0.0, 0.9, n_tpl) * rng.uniform(0.05, 1.0)
        sets = [set(np.flatnonzero(rng.random(n_tpl) < p).tolist()) for _ in range(F)]
        n_kp_global = int(rng.choice([1, 5, 10, 50, 100, 500]))
        kb = _bits(sets, n_tpl)
        cuts = sorted({0, F, *rng.integers(0, F + 1, int(rng.integers(0, 4))).tolist()})
        try:
            cons_set, order, votes = oracle.consensus(sets, n_kp_global, 1)
        except RuntimeError:
            continue
        choice, po, pi = _split_consensus(kb, n_tpl, n_kp_global, 1, cuts)
        assert choice.order.tolist() == list(order) and choice.votes.tolist() == list(votes)
        assert choice.cons_iter.tolist() == list(cons_set)
        lists = oracle.lookup(cons_set, sets)
        for f, L in enumerate(lists):
            assert pi[po[f]:po[f + 1]].tolist() == L
        full = stages.consensus(kb, n_tpl, n_kp_global, 1)
        assert np.array_equal(full.pt_off, po) and np.array_equal(full.pt_idx, pi)


def test_consensus_vote_first_occurrence_keys():
    """The vote's key row: (frame << 32) | slot of the template in the first frame's set
    table (iteration position), INT64_MAX for templates no frame holds."""
    sets = [set(), {5, 3, 900}, {3, 7}, {1000 % 1001}]
    kb = _bits(sets, 1001)
    v = stages.consensus_vote_host(kb, 1001, frame_base=10)
    assert v[0, 3] == 2 and v[0, 7] == 1 and v[0, 999] == 0
    assert v[1, 999] == np.iinfo(np.int64).max
    assert v[1, 3] >> 32 == 11 and v[1, 7] >> 32 == 12 and v[1, 1000] >> 32 == 13
    it = list({5, 3, 900})  # CPython's iteration order of frame 1's set
    slots = sorted((v[1, k] & 0xFFFFFFFF, k) for k in (3, 5, 900))
    assert [k for _, k in slots] == it


def test_consensus_merge_too_few_raises_and_bad_votes():
    v = stages.consensus_vote_host(_bits([{1, 2}, {2, 3}], 10), 10)
    with pytest.raises(VideoAligner.AlignmentError):
        stages.consensus_merge(v, 10, 10, 5)
    bad = v.copy()
    bad[1, 2] = np.iinfo(np.int64).max  # a voted template without a first occurrence
    with pytest.raises(ValueError):
        stages.consensus_merge(bad, 10, 10, 1)


# ------------------------------------------------------------ sharded gap filling
@pytest.mark.parametrize("lerp", [True, False])
def test_fill_gaps_slab_equals_global_interpolation(lerp):
    """affines.fill_gaps_slab on every rank's slab with only its two neighbouring models ==
    the rows of the global interpolate_affines / interpolate_linear, incl. gaps that span
    whole ranks and leading / trailing gaps."""
    from kcmc_amd import distributed as kdist

    rng = np.random.default_rng(4 if lerp else 5)
    for case in range(60):
        n = int(rng.integers(2, 40))
        t = rng.normal(0, 0.05, n)
        a = np.stack([np.array([[np.cos(x), -np.sin(x), rng.normal()], [np.sin(x), np.cos(x), rng.normal()]]) for x in t])
        miss = rng.random(n) < rng.choice([0.1, 0.5, 0.9])
        if case % 7 == 0:
            miss[: n // 2] = True
        if miss.all():
            miss[int(rng.integers(0, n))] = False
        a[miss] = np.nan
        ref, ref_it = (affines.interpolate_affines if lerp else affines.interpolate_linear)(a)
        ref_sk = np.flatnonzero(miss).tolist()
        cuts = sorted({0, n, *rng.integers(0, n + 1, int(rng.integers(0, 5))).tolist()})
        counts = [b - c for c, b in zip(cuts, cuts[1:])]
        bounds = []
        for c, b in zip(cuts, cuts[1:]):
            ok = np.flatnonzero(~miss[c:b])
            row = np.full(14, np.nan)
            row[:2] = (ok[0], ok[-1]) if ok.size else (-1, -1)
            if ok.size:
                row[2:8], row[8:] = a[c + ok[0]].ravel(), a[c + ok[-1]].ravel()
            bounds.append(row)
        bounds = np.stack(bounds)
        got, sk, it = [], [], []
        for r, (c, b) in enumerate(zip(cuts, cuts[1:])):
            prev, nxt = kdist.neighbours(bounds, counts, r)
            m, s, i = affines.fill_gaps_slab(a[c:b], c, prev, nxt, lerp)
            got.append(m)
            sk += s
            it += i
        np.testing.assert_array_equal(np.concatenate(got), ref)
        assert sk == ref_sk and it == ref_it
    with pytest.raises(VideoAligner.AlignmentError):
        affines.fill_gaps_slab(np.full((3, 2, 3), np.nan), 4, None, None, True)


def _square_plus(i, x, k=0):  # module level: picklable for the process pool
    return i * 1000 + x * x + k


def test_parallelize_is_an_ordered_process_pool_map():
    """VA:460-471: _parallelize / _parallelize_i map a picklable per-frame function over equal
    sequences in a joblib multiprocessing pool of N_JOBS_PARALLEL workers, results in order;
    one worker (or this package's own GPU-backed functions) runs in this process."""
    va = VideoAligner()
    xs = list(range(37))
    assert va._parallelize_i(_square_plus, xs, k=5) == [i * 1000 + i * i + 5 for i in xs]

    class One(VideoAligner):
        N_JOBS_PARALLEL = 1

    assert One()._parallelize(_square_plus, [1, 2], [3, 4]) == [1009, 2016]


@pytest.mark.parametrize("counts", [[3, 3, 3], [3, 0, 2], [0, 0], []])
def test_keypoints_csr_compacts_in_frame_order(counts):
    """stages.keypoints_csr: the first count[f] detections of every frame, frame by frame
    (the matcher's CSR), whether every frame is full or not."""
    import torch

    F, N = len(counts), 3
    kp = torch.arange(F * N * 2, dtype=torch.float64).reshape(F, N, 2)
    des = torch.arange(F * N * 32, dtype=torch.int64).remainder(251).to(torch.uint8).reshape(F, N, 32)
    k = stages.Keypoints(kp, des, torch.tensor(counts, dtype=torch.int32))
    kp_q, des_q, q_off, q_off_host = stages.keypoints_csr(k)
    rows = [(f, j) for f in range(F) for j in range(counts[f])]
    assert q_off_host.tolist() == [0] + np.cumsum(counts).astype(int).tolist()
    assert q_off.tolist() == q_off_host.tolist()
    assert kp_q.shape == (len(rows), 2) and des_q.shape == (len(rows), 32)
    for i, (f, j) in enumerate(rows):
        assert kp_q[i].tolist() == kp[f, j].tolist()
        assert des_q[i].tolist() == des[f, j].tolist()
