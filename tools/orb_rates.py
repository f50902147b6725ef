"""Detection (f1, csrc/orb.hip) rate at the bench's 1080p shape with an output digest, for
same-box A/B of library builds (KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/<name>.so):

    python tools/orb_rates.py [--frames 2000] [--reps 5]

The stack is bench.py's c2 frames (the texture seen through each frame's jitter) scaled
to u8; stages.detect_orb is timed with HIP events around each call.  Prints one JSON
line: median / best ms, frames per second and a digest of (keypoints, descriptors,
counts), which must agree between builds."""
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
from kcmc_amd import stages  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bc = bench.CONFIGS["c2"]
    inp, _ = bench.make_inputs(bc, a.frames, 0, dev)
    u8 = stages.max_scale_u8(inp.frames, stages.brightest_px(inp.frames))
    del inp
    k = stages.detect_orb(u8)
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        k = stages.detect_orb(u8)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    h = hashlib.sha1()
    cnt = k.count.cpu().numpy()
    h.update(cnt.tobytes())
    kp, des = k.kp.cpu().numpy(), k.des.cpu().numpy()
    for f in range(len(cnt)):
        h.update(kp[f, :cnt[f]].tobytes())
        h.update(des[f, :cnt[f]].tobytes())
    med = float(np.median(ts))
    print(json.dumps({"lib": os.environ.get("KCMC_LIB_PATH", "in-tree"), "frames": a.frames, "ms_median": round(med, 3),
                      "ms_best": round(min(ts), 3), "frames_per_s": round(a.frames / med * 1e3, 1),
                      "mean_keypoints": float(cnt.mean()), "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
