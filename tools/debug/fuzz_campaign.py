"""A longer run of the seeded fuzz sweeps of tests/test_gpu_fuzz.py (bug hunting on the GPU
box, not part of the suite): every test function over seeds [start, start + n), failures
printed with their seed so they can be pinned as a regular test case.

    python tools/debug/fuzz_campaign.py <n> [start] [name-filter]
"""
import os
import sys
import time
import traceback

import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "oracle"), os.path.join(R, "tests")]
import kcmc_amd  # noqa: E402,F401
import test_gpu_fuzz as T  # noqa: E402

n = int(sys.argv[1])
start = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
filt = sys.argv[3] if len(sys.argv) > 3 else ""
dev = torch.device("cuda", 0)
cases = [("warp", lambda s: T.test_warp_fuzz_vs_oracle(dev, s)),
         ("knn_l2u8", lambda s: T.test_knn2_fuzz_vs_oracle(dev, "l2u8", s)),
         ("knn_hamming", lambda s: T.test_knn2_fuzz_vs_oracle(dev, "hamming", s)),
         ("knn_l2f32", lambda s: T.test_knn2_fuzz_vs_oracle(dev, "l2f32", s)),
         ("ransac_rigid", lambda s: T.test_ransac_rigid_fuzz_vs_oracle(dev, s)),
         ("ransac_affine", lambda s: T.test_ransac_model_fuzz_vs_oracle(dev, "affine", s)),
         ("ransac_projective", lambda s: T.test_ransac_model_fuzz_vs_oracle(dev, "projective", s)),
         ("filters", lambda s: T.test_match_filters_fuzz_vs_oracle(dev, s)),
         ("slab", lambda s: T.test_slab_end_to_end_fuzz_vs_oracle(dev, s)),
         ("pyr_norm", lambda s: T.test_pyr_down_and_normalize_fuzz(dev, s)),
         ("orb", lambda s: T.test_orb_detect_fuzz_vs_oracle(dev, s)),
         ("split", lambda s: T.test_multidevice_split_fuzz(dev, s)),
         ("overlapped", lambda s: T.test_overlapped_slabs_fuzz(dev, s))]
def knn_large(kind, seed):
    """The matchers at config-4/5 sizes: n_tpl up to 6000, frames up to 5000 rows, D up to the
    limit, exact template copies among the rows (ties), a few frames of 2 rows."""
    import numpy as np

    import oracle
    from kcmc_amd import stages

    rng = np.random.default_rng(50000 + seed)
    if kind == "l2f32":
        D = int(rng.choice([64, 100, 128]))
        gen = lambda n: rng.normal(0, 1.0, (n, D)).astype(np.float32)  # noqa: E731
    else:
        D = int(rng.choice([32, 61, 64]))
        gen = lambda n: rng.integers(0, 256, (n, D), dtype=np.uint8)  # noqa: E731
    n_tpl = int(rng.integers(1000, 6001))
    tpl = gen(n_tpl)
    frames = []
    for _ in range(int(rng.integers(1, 4))):
        n_q = int(rng.choice([2, int(rng.integers(1000, 5001))]))
        q = gen(n_q)
        k = n_q // 3
        q[:k] = tpl[rng.integers(0, n_tpl, k)]
        frames.append(q)
    off = np.zeros(len(frames) + 1, np.int32)
    off[1:] = np.cumsum([len(q) for q in frames])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    fn = stages.knn2_hamming if kind == "hamming" else stages.knn2_l2u8
    idx, dist = fn(t(tpl), t(np.concatenate(frames)), t(off), int(np.diff(off).max()))
    idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
    ora = {"l2u8": oracle.knn2_l2u8, "hamming": oracle.knn2_hamming, "l2f32": oracle.knn2_l2f32}[kind]
    for f, q in enumerate(frames):
        ri, rd = ora(tpl, q)
        assert np.array_equal(idx[f], ri), (kind, seed, f, n_tpl, len(q), D)
        assert np.array_equal(dist[f].view(np.int32), rd.view(np.int32)), (kind, seed, f)


def warp_large(seed):
    """The warp at config sizes (1080p / 4K, C = 1 / 3 / 4, 1-2 frames) with the sweep's map
    families, affine and perspective, forward and inverse."""
    import numpy as np

    import oracle
    from kcmc_amd import stages

    rng = np.random.default_rng(60000 + seed)
    H, W = [(1080, 1920), (2160, 3840), (1079, 1917)][int(rng.integers(0, 3))]
    C = int(rng.choice([1, 3, 4]))
    F = int(rng.integers(1, 3))
    shape = (F, H, W) if C == 1 else (F, H, W, C)
    imgs = T._values(rng, shape)
    persp = bool(rng.integers(0, 2))
    Ms = np.stack([(T._perspective if persp else T._affine)(rng, H, W) for _ in range(F)])
    inv = bool(rng.integers(0, 2))
    fn = stages.warp_perspective_u16 if persp else stages.warp_affine_u16
    ref = oracle.warp_perspective_u16 if persp else oracle.warp_affine_u16
    out = fn(torch.from_numpy(imgs).to(dev), torch.from_numpy(Ms).to(dev), inverse_map=inv).cpu().numpy()
    for f in range(F):
        assert np.array_equal(out[f], ref(imgs[f], Ms[f], inverse_map=inv)), (seed, shape, persp, inv, f)


cases += [("large_warp", warp_large)]
cases += [("large_knn_l2u8", lambda s: knn_large("l2u8", s)), ("large_knn_hamming", lambda s: knn_large("hamming", s)),
          ("large_knn_l2f32", lambda s: knn_large("l2f32", s))]
fails = 0
for name, fn in cases:
    if filt and filt not in name:
        continue
    t0 = time.time()
    bad = []
    for s in range(start, start + n):
        if (s - start) % 250 == 249:
            print(f"  {name}: {s - start + 1}/{n} ({len(bad)} failed, {time.time() - t0:.0f} s)", flush=True)
        try:
            fn(s)
        except Exception as e:  # noqa: BLE001 - report and go on
            bad.append(s)
            print(f"FAIL {name} seed {s}: {type(e).__name__}: {str(e)[:300]}", flush=True)
            if len(bad) == 1:
                traceback.print_exc()
    fails += len(bad)
    print(f"{name}: {n - len(bad)}/{n} ok in {time.time() - t0:.1f} s", flush=True)
print(f"total failures: {fails}")
sys.exit(1 if fails else 0)
