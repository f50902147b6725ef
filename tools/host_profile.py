"""cProfile of the host side of the pipelined bench step (OverlappedSlabs.submit):
which Python / torch / ctypes calls make up the per-step host chain.

    python tools/host_profile.py [--config c3] [--steps 40] [--top 45]

Prints the step time with and without the profiler, then the top functions by own time
and by cumulative time (per step, microseconds)."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from kcmc_amd import pipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--top", type=int, default=45)
    args = ap.parse_args()
    bc = bench.CONFIGS[args.config]
    frames = args.frames or bc.frames_per_gpu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    inp, _ = bench.make_inputs(bc, frames, 0, dev)
    out = torch.empty_like(inp.frames)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=bc.match_beside)

    def run(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            ov.submit(inp, out=out)
        ov.flush()
        ov.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n

    run(5)
    plain = run(args.steps)
    pr = cProfile.Profile()
    pr.enable()
    prof = run(args.steps)
    pr.disable()
    print(f"config {args.config} frames {frames}: step {plain:.3f} ms (profiled {prof:.3f} ms)")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        st = pstats.Stats(pr, stream=s)
        st.sort_stats(key).print_stats(args.top)
        print(f"==== by {key} (totals over {args.steps} steps) ====")
        print(s.getvalue())


if __name__ == "__main__":
    main()
