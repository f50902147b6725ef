"""Isolated RANSAC stage time at a bench config's shape, with an output digest for
same-box A/B of library builds (KCMC_LIB_PATH=ab/<name>.so, see tools/ab_build.py):

    python tools/ransac_rates.py [--config c2] [--reps 10]

Keypoints, match and consensus come from bench.py's own generator (no frames are
warped); the RANSAC stage (VA:137-142) is timed with HIP events around `reps` calls
after one warm-up call.  Prints one JSON line: median / best ms, hypotheses per second
and a digest of (params, inliers, n_inliers, best trial), which must agree between
builds."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from kcmc_amd import pipeline, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--device-lists", action="store_true",
                    help="the pipelines' form: device consensus lists (kcmc_ransac_lists, max_n = n_kp_global)")
    a = ap.parse_args()
    bc = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    ks = synthetic.make_keypoints(bc.frames_per_gpu, bc.n_tpl, bc.D, (bc.H, bc.W), seed=3, frame_seed=0,
                                  model=bc.model, descriptor=bc.descriptor)
    inp = pipeline.SlabInputs(None, torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                              torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                              torch.from_numpy(ks.q_off).to(dev), ks.q_off)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    m = pipeline.match_stage(inp, cfg)
    if a.device_lists:
        cons = pipeline.device_consensus(m, bc.n_tpl, bc.frames_per_gpu, cfg)
        lists = None
    else:
        keep = m.keep_bits.cpu().numpy()
        cons = pipeline.consensus_stage(keep, bc.n_tpl, keep.shape[0], cfg)
        lists = pipeline.consensus_to_device(cons, dev)
    rr = pipeline.ransac_stage(m, inp.kp_tpl, cons, cfg, lists_dev=lists)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rr = pipeline.ransac_stage(m, inp.kp_tpl, cons, cfg, lists_dev=lists)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    h = hashlib.sha1()
    for t in (rr.params, rr.inliers, rr.n_inliers, rr.best_trial):
        h.update(np.ascontiguousarray(t.cpu().numpy()).tobytes())
    n_fit = int((np.diff(cons.pt_off) >= cfg.effective_frame_skip).sum())
    med = float(np.median(ts))
    print(json.dumps({"config": a.config, "lists": "device" if a.device_lists else "host", "lib": os.environ.get("KCMC_LIB_PATH", "in-tree"), "frames": bc.frames_per_gpu,
                      "frames_fitted": n_fit, "mean_points": float(np.diff(cons.pt_off).mean()),
                      "ms_median": round(med, 4), "ms_best": round(min(ts), 4),
                      "hypotheses_per_s": round(n_fit * cfg.ransac_trials / (med * 1e-3), 1),
                      "digest": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main()
