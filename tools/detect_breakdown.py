"""Where the time of bench.py's `with_detection` pass goes (config 2: 2000 x 1080p on one
MI355X): each stage of pipeline.detect_slab / align_slab timed with a device sync on
both sides.  Prints one JSON object (ms per stage, best of `--reps`)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcmc_amd import pipeline, stages, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    F, H, W = args.frames, 1080, 1920
    base = torch.from_numpy(synthetic.make_texture((H, W), seed=0)).to(dev)
    frames = base[None].expand(F, H, W).contiguous()
    cfg = pipeline.AlignConfig(n_kp_global=100)
    best = {}

    def t(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0)
        best[name] = min(best.get(name, ms), ms)
        return r

    for _ in range(args.reps):
        b = t("percentile", lambda: stages.brightest_px(frames))
        u8 = t("max_scale", lambda: stages.max_scale_u8(frames, b))
        tpl = u8[F // 2:F // 2 + 1]
        kt = t("detect_template", lambda: stages.detect_orb(tpl))
        kq = t("detect_frames", lambda: stages.detect_orb(u8))
        n_t = int(kt.count.cpu()[0])
        kp_q, des_q, q_off, q_off_host = t("keypoints_csr", lambda: stages.keypoints_csr(kq))
        inp = pipeline.SlabInputs(frames, kt.des[0, :n_t].contiguous(), kt.kp[0, :n_t].contiguous(), des_q, kp_q,
                                  q_off, q_off_host)
        out = torch.empty_like(frames)
        t("align_slab", lambda: pipeline.align_slab(inp, cfg, out=out))
        t("align_frames_total", lambda: pipeline.align_frames(frames, cfg, out=out))
    best = {k: round(v, 3) for k, v in best.items()}
    best["sum_of_stages"] = round(sum(v for k, v in best.items() if k != "align_frames_total"), 3)
    print(json.dumps(best))


if __name__ == "__main__":
    main()
