"""Host timeline of the overlapped bench step (bench.py's workloads, default c2): where the
host spends a step while the warp of the previous step runs on the GPU.

    python tools/host_breakdown.py [--config c2] [--frames F] [--steps 8]

Prints, per step, host wall-clock milliseconds between the marks OverlappedSlabs.submit
passes through (m0 match(k) launched, m1, w0/w1 around the warp(k-2) launch, r0 after
the bitmask wait + native consensus of slab k-1, r1 its RANSAC launched, end after the
post-processing of slab k-2), and the consensus alone on the same bitmasks.  The device
idles when the host's chain outlasts the step's kernels."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kcmc_amd import pipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    bc = bench.CONFIGS[args.config]
    args.frames = args.frames or bc.frames_per_gpu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    inp, _ = bench.make_inputs(bc, args.frames, 0, dev)
    out = torch.empty_like(inp.frames)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    ov = pipeline.OverlappedSlabs(dev, cfg, match_beside=bc.match_beside)
    rows = []
    for s in range(args.steps + 2):
        if s == 2:
            ov.synchronize()
            t_start = time.perf_counter()
        t = {}
        t0 = time.perf_counter()
        ov.submit(inp, out=out, mark=lambda n, ev=None: t.__setitem__(n, time.perf_counter()))
        t["end"] = time.perf_counter()
        if s >= 2:
            keys = ["m0", "m1", "w0", "w1", "r0", "r1", "end"]
            rows.append({f"{a}->{b}": round((t[b] - t[a]) * 1e3, 3) for a, b in zip(keys, keys[1:])}
                        | {"submit_ms": round((t["end"] - t0) * 1e3, 3)})
    ov.flush()
    ov.synchronize()
    step_ms = (time.perf_counter() - t_start) * 1e3 / args.steps
    keep = pipeline.match_stage(inp, cfg).keep_bits.cpu().numpy()
    cons = []
    for _ in range(5):
        c0 = time.perf_counter()
        pipeline.consensus_stage(keep, inp.des_tpl.shape[0], args.frames, cfg, None)
        cons.append((time.perf_counter() - c0) * 1e3)
    med = {k: round(float(np.median([r[k] for r in rows])), 3) for k in rows[0]}
    sub = np.array([r["submit_ms"] for r in rows])
    pct = {p: round(float(np.percentile(sub, p)), 3) for p in (10, 50, 90, 99)}
    slow = [(i, {k: v for k, v in r.items() if v > 2 * med[k] + 0.05}) for i, r in enumerate(rows)
            if r["submit_ms"] > 1.5 * med["submit_ms"]]
    print(json.dumps({"config": args.config, "frames": args.frames, "step_ms": round(step_ms, 3), "median_host_ms": med, "submit_ms_percentiles": pct, "slow_submits": slow[:12], "consensus_alone_ms": round(min(cons), 3),
                      "cpu_count": os.cpu_count()}))


if __name__ == "__main__":
    main()
