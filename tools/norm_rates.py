"""The normalisation front end (f2, csrc/normalize.hip) at the bench's 1080p shape, for
same-box A/B of library builds (KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/<name>.so):
stages.brightest_px (the two histogram passes + the host interpolation) and
stages.max_scale_u8, timed with a device sync on both sides; prints one JSON line with the
percentile value and a digest of the u8 stack, which must agree between builds."""
import argparse
import hashlib
import json
import os
import sys
import time

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
    inp, _ = bench.make_inputs(bench.CONFIGS["c2"], a.frames, 0, dev)
    fr = inp.frames
    del inp

    def timed(fn):
        ts, r = [], None
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        return float(np.median(ts[1:])), r

    ms_p, b = timed(lambda: stages.brightest_px(fr))
    ms_s, u8 = timed(lambda: stages.max_scale_u8(fr, b))
    h = hashlib.sha1(u8.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.environ.get("KCMC_LIB_PATH", "in-tree"), "frames": a.frames,
                      "percentile_ms": round(ms_p, 3), "max_scale_ms": round(ms_s, 3), "brightest": float(b),
                      "u8_digest": h}), flush=True)


if __name__ == "__main__":
    main()
