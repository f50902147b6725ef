"""Per-kernel rates of the section-8f rows on one MI355X, with the
roofline each is priced against.  Prints one JSON object.

    python tools/kernel_rates.py [--frames 2000]

Inputs are device-resident synthetic stacks (the bench texture, kcmc_amd.synthetic);
every timing is HIP events around `reps` launches on the current stream after one
warmup launch.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcmc_amd import stages, synthetic  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X datasheet (MI355X_MICROARCH.md)


def timed(fn, reps):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def stack(F, H, W, dev):
    base = torch.from_numpy(synthetic.make_texture((H, W), seed=0)).to(dev)
    return base[None].expand(F, H, W).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    F, H, W = args.frames, 1080, 1920
    out = {"device": torch.cuda.get_device_name(0), "frames": F}

    frames = stack(F, H, W, dev)
    n = frames.numel()
    hist = torch.empty(256, dtype=torch.int64, device=dev)
    from kcmc_amd import _lib
    L, ctx = _lib.load(), stages._ctx(dev).handle

    def hist_pass():
        _lib.check(L.kcmc_histogram_u16(ctx, stages._ptr(frames), n, 8, -1, stages._ptr(hist), stages._stream(dev)))

    ms = timed(hist_pass, args.reps)
    out["f2_histogram_u16"] = {"ms": ms, "bytes": 2 * n, "GBps": 2 * n / ms / 1e6, "frac": 2 * n / ms / 1e6 / HBM_PEAK_GBPS,
                               "unit": "one 256-bin pass over F x 1080 x 1920 u16"}
    ms = timed(lambda: stages.brightest_px(frames), max(1, args.reps // 2))
    out["f2_percentile_total"] = {"ms": ms, "note": "coarse + fine histogram passes + host interpolation"}
    u8 = torch.empty(frames.shape, dtype=torch.uint8, device=dev)
    ms = timed(lambda: stages.max_scale_u8(frames, 39116.8, out=u8), args.reps)
    out["f2_lut_u16_to_u8"] = {"ms": ms, "bytes": 3 * n, "GBps": 3 * n / ms / 1e6, "frac": 3 * n / ms / 1e6 / HBM_PEAK_GBPS}
    del frames

    # f4 pyrDown: LoResVideoAligner on square frames (config 3's 512^2 two-photon stack)
    Fs = 8 * F
    sq = stack(Fs, 512, 512, dev)
    sq8 = stages.max_scale_u8(sq, 39116.8)
    del sq
    pd = torch.empty((Fs, 256, 256), dtype=torch.uint8, device=dev)
    ms = timed(lambda: stages.pyr_down_u8(sq8, (256, 256), out=pd), args.reps)
    nb = sq8.numel() * 1.25
    out["f4_pyr_down_u8"] = {"ms": ms, "frames": Fs, "shape": [512, 512], "bytes": nb, "GBps": nb / ms / 1e6,
                             "frac": nb / ms / 1e6 / HBM_PEAK_GBPS, "unit": "1 B read + 0.25 B written per source px"}
    del sq8, pd

    # f1 detection on the u8 1080p stack
    Fd = min(F, 500)
    ms = timed(lambda: stages.detect_orb(u8[:Fd]), max(1, args.reps // 2))
    out["f1_detect_orb"] = {"ms": ms, "frames": Fd, "frames_per_s": Fd / ms * 1e3,
                            "GBps_input": u8[:Fd].numel() / ms / 1e6}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
