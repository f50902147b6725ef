"""Phase breakdown of the rigid RANSAC scorer from the stamp build (tools/ab_patches/
ransac_stamps.py): per frame, the shader cycles between the barriers that end each phase,
the workgroups' start times (how many rounds of resident workgroups the launch takes) and
the phase A2 / phase B work counts.

    KCMC_AB_PATCH=tools/ab_patches/ransac_stamps.py python tools/ab_build.py stamps
    KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/stamps.so python tools/debug/ransac_stamps.py [--config c2]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

NAMES = ["staging", "phase A", "phase A2", "best count", "phase B+argmax", "selection", "mask+refit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    from kcmc_amd import _lib, pipeline

    bc = bench.CONFIGS[a.config]
    if bc.model != "euclidean":
        raise SystemExit("the stamp build instruments the rigid scorer only")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    inp, _ = bench.make_inputs(bc, bc.frames_per_gpu, 0, dev)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    n_tpl = inp.des_tpl.shape[0]
    F = inp.q_off.numel() - 1
    m = pipeline.match_stage(inp, cfg)
    cons = pipeline.device_consensus(m, n_tpl, F, cfg)
    times = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pipeline.ransac_stage(m, inp.kp_tpl, cons, cfg)
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    st = np.zeros((F, 12), np.uint64)
    L = _lib.load()
    if L.kcmc_debug_ransac_stamps(ctypes.c_void_p(st.ctypes.data), ctypes.c_int(F)) != 0:
        raise SystemExit("kcmc_debug_ransac_stamps failed (not the stamp build?)")
    s = st.astype(np.int64)
    ok = s[:, 7] != 0
    print(f"{a.config}: {F} frames, {int(ok.sum())} scored; stage {np.median(times):.4f} ms median of {a.reps} "
          f"(events, last launch's stamps)")
    s0 = s[ok, 0] - s[ok, 0].min()
    span = (s[ok, 7].max() - s[ok, 0].min())
    print(f"  launch span {span} cycles; workgroup start offsets: "
          + ", ".join(f"p{q} {int(np.percentile(s0, q))}" for q in (0, 25, 50, 75, 90, 100)))
    fast = ok & (s[:, 2] != 0)
    seq = [0, 1, 2, 3, 4, 5, 6, 7]
    tot = (s[ok, 7] - s[ok, 0])
    print(f"  per frame total: mean {tot.mean():.0f}, median {np.median(tot):.0f}, p90 {np.percentile(tot, 90):.0f} cycles")
    for i, n in enumerate(NAMES):
        a_, b_ = seq[i], seq[i + 1]
        rows = fast if a_ in (1, 2) or b_ in (2, 3) else ok
        d = s[rows, b_] - s[rows, a_]
        print(f"  {n:16s} mean {d.mean():8.0f}  median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  "
              f"share {d.mean() / tot.mean():.3f}")
    print(f"  A2 trials per frame: mean {s[ok, 8].mean():.2f}, max {s[ok, 8].max()}; phase-B candidates: mean "
          f"{s[ok, 9].mean():.2f}, max {s[ok, 9].max()}; exact-path frames {int(s[ok, 10].sum())}; "
          f"fp32-path frames {int(fast.sum())}")
    # start-time clusters: workgroups that start within the first 5 % of the span are round 1
    r1 = s0 < 0.05 * span
    print(f"  workgroups starting in the first 5 % of the span: {int(r1.sum())}; their mean total "
          f"{tot[r1].mean():.0f}, the rest {tot[~r1].mean() if (~r1).any() else 0:.0f} cycles")


if __name__ == "__main__":
    main()
