"""Isolated rates of the K1 matchers at each BASELINE config's matching shape, with the
MFMA roofline each is priced against.  Prints one JSON object.

    python tools/match_rates.py [--configs c2,c3,c4,c5] [--reps 5]

Per config: F frames of synthetic keypoints (kcmc_amd.synthetic, the bench's
generator), `kcmc_knn2_l2u8` (uint8, int8 MFMA) or `kcmc_knn2_l2f32` (float, bf16x3
MFMA + fp64 re-rank) timed with HIP events around `reps` launches on the current
stream after one warm-up launch.  Algorithmic work = 2 * n_tpl * n_q * D per frame
(int ops for uint8, flops for float32); peaks from MI355X_MICROARCH.md: I8 dense
~5.0 POPS (2x the bf16 rate), BF16 dense ~2.5 PF (the float matcher issues three bf16
products per fp32 product, so it is priced against bf16 / 3 for its fp32-equivalent
work and against bf16 for its issued MFMA work).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcmc_amd import stages, synthetic  # noqa: E402

I8_PEAK_TOPS = 5000.0
BF16_PEAK_TFLOPS = 2500.0

# (frames, n_tpl, D, descriptor, H, W): the match stage of each bench config
SHAPES = {
    "c2": (2000, 500, 32, "u8", 1080, 1920),
    "c3": (2500, 500, 61, "u8", 512, 512),
    "c4": (625, 4096, 61, "u8", 2160, 3840),
    "c5": (500, 4096, 128, "f32", 1080, 1920),
    # the opt-in NORM_HAMMING matcher on c2's shape (VALU popcount, priced against the
    # VALU issue rate: 2 * D/4 + 3 instructions per distance)
    "c2h": (2000, 500, 32, "hamming", 1080, 1920),
}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {"device": torch.cuda.get_device_name(0)}
    for name in args.configs.split(","):
        F, n_tpl, D, desc, H, W = SHAPES[name]
        ks = synthetic.make_keypoints(F, n_tpl, D, (H, W), seed=3, frame_seed=0,
                                      descriptor="u8" if desc == "hamming" else desc)
        tpl = torch.from_numpy(ks.des_tpl).to(dev)
        q = torch.from_numpy(ks.des_q).to(dev)
        off = torch.from_numpy(ks.q_off).to(dev)
        max_nq = int(np.diff(ks.q_off).max())
        knn = stages.knn2_hamming if desc == "hamming" else stages.knn2_l2u8  # l2u8 dispatches on dtype
        ms = timed(lambda: knn(tpl, q, off, max_nq), args.reps)
        ops = 2.0 * n_tpl * float(ks.q_off[-1]) * D
        rate = ops / (ms * 1e-3) / 1e12
        r = {"frames": F, "n_tpl": n_tpl, "D": D, "descriptor": desc, "mean_n_q": round(ks.q_off[-1] / F, 1),
             "ms": round(ms, 4), "algorithmic_ops": ops}
        if desc == "hamming":
            d = n_tpl * float(ks.q_off[-1])
            r.update({"G_distances_per_s": round(d / (ms * 1e-3) / 1e9, 1)})
        elif desc == "f32":
            r.update({"TFLOPs_fp32_equiv": round(rate, 1), "bf16_mfma_TFLOPs_issued": round(3 * rate, 1),
                      "peak": BF16_PEAK_TFLOPS, "frac_bf16_issued": round(3 * rate / BF16_PEAK_TFLOPS, 4)})
        else:
            r.update({"TOPs": round(rate, 1), "peak": I8_PEAK_TOPS, "frac": round(rate / I8_PEAK_TOPS, 4)})
        out[name] = r
        print(name, r, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
