"""Time the REFERENCE's own RANSAC stage next to the CPU port that bench.py's cpu_baseline
times, on the same host and the same inputs (build container only: the reference and
scikit-image 0.18.3 are not on the GPU box).

    /opt/conda/bin/python3.9 tools/reference_cpu_calibration.py [--frames 240] [--procs 8] [--n 90]

Reference: /root/reference/VideoAligner.py imported with a stub ``cv2`` module (only the
detector constructors the class body references, VA:22-25; nothing cv2 runs here), then
    VideoAligner()._parallelize(VideoAligner._compute_euclidean_affine, kp_template_list,
                              kp_query_list, spatial_downsample_rate=1)           (VA:137-142)
exactly as align_images calls it: joblib multiprocessing over N_JOBS_PARALLEL processes,
skimage 0.18.3 ransac(EuclideanTransform, 2, 2, 1000 trials, random_state=42) per frame.
Port: the oracle's numpy/LAPACK restatement of the same call (oracle.ransac_rigid_skimage,
what cpu_baseline_workers.py runs per frame) in a pool of the same size.
Inputs: BASELINE config-2-like point lists (N consensus points per frame, 1080p template
coordinates, a rigid jitter, 0.3 px noise, 20 % outliers), seeded.
Writes profiles/r03_cpu_reference_calibration.json."""
import argparse
import importlib.util
import json
import multiprocessing as mp
import os
import sys
import time
import types
import warnings

import numpy as np

warnings.filterwarnings("ignore")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/VideoAligner.py"


def _load_reference():
    cv2 = types.ModuleType("cv2")
    cv2.AKAZE_create = object
    cv2.BRISK_create = object
    sys.modules["cv2"] = cv2
    spec = importlib.util.spec_from_file_location("VideoAligner", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["VideoAligner"] = mod  # joblib pickles the static methods by module name
    spec.loader.exec_module(mod)
    return mod.VideoAligner


def _inputs(F, N, seed=0):
    rng = np.random.default_rng(seed)
    tpl, qry = [], []
    for _ in range(F):
        t = rng.uniform(0, (1920, 1080), (N, 2))
        th, tx, ty = rng.normal(0, np.deg2rad(0.5)), rng.normal(0, 4), rng.normal(0, 4)
        c, s = np.cos(th), np.sin(th)
        # frame -> template map is the jitter; the frame points are its inverse image
        q = (t - (tx, ty)) @ np.array([[c, -s], [s, c]])
        q += rng.normal(0, 0.3, q.shape)
        out = rng.random(N) < 0.2
        q[out] = rng.uniform(0, (1920, 1080), (int(out.sum()), 2))
        tpl.append(t)
        qry.append(q)
    return tpl, qry


_P = {}


def _port_init():
    from threadpoolctl import threadpool_limits

    threadpool_limits(1)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    _P["o"] = oracle


def _port_chunk(items):
    o = _P["o"]
    return [o.ransac_rigid_skimage(q, t)[0] for t, q in items]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--n", type=int, default=90)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03_cpu_reference_calibration.json"))
    args = ap.parse_args()
    VA = _load_reference()
    VA.N_JOBS_PARALLEL = args.procs
    va = VA()
    tpl, qry = _inputs(args.frames, args.n)

    # the reference: its own _parallelize over its own static method (warm-up on a few frames first)
    va._parallelize(VA._compute_euclidean_affine, tpl[:args.procs], qry[:args.procs], spatial_downsample_rate=1)
    t0 = time.perf_counter()
    ref = va._parallelize(VA._compute_euclidean_affine, tpl, qry, spatial_downsample_rate=1)
    t_ref = time.perf_counter() - t0

    # the port, same pool size, frames in contiguous chunks like cpu_baseline_workers.py
    chunks = [list(zip(tpl[i::args.procs], qry[i::args.procs])) for i in range(args.procs)]
    with mp.get_context("spawn").Pool(args.procs, initializer=_port_init) as pool:
        pool.map(_port_chunk, [c[:1] for c in chunks])
        t0 = time.perf_counter()
        port = pool.map(_port_chunk, chunks)
        t_port = time.perf_counter() - t0
    port_by_frame = {}
    for i, c in enumerate(port):
        for k, p in enumerate(c):
            port_by_frame[i + k * args.procs] = p
    diff = max(float(np.nanmax(np.abs(port_by_frame[f] - ref[f]) / np.maximum(np.abs(ref[f]), 1.0)))
               for f in range(args.frames))
    res = {
        "host": f"build container, {os.cpu_count()} CPUs",
        "inputs": f"{args.frames} frames, N = {args.n} consensus points each (config-2-like rigid jitter, 0.3 px noise, "
                  f"20 % outliers), 1000 trials",
        "procs": args.procs,
        "reference": {"what": "VideoAligner._parallelize(VideoAligner._compute_euclidean_affine, ...) (VA:137-142, "
                              "VA:460-465) with scikit-image 0.18.3, stub cv2 import",
                      "seconds": round(t_ref, 3), "frames_per_s": round(args.frames / t_ref, 2),
                      "ms_per_frame_per_core": round(1e3 * t_ref * args.procs / args.frames, 2)},
        "port": {"what": "oracle.ransac_rigid_skimage (numpy/LAPACK restatement; cpu_baseline's RANSAC) in a "
                         "spawn pool of the same size",
                 "seconds": round(t_port, 3), "frames_per_s": round(args.frames / t_port, 2),
                 "ms_per_frame_per_core": round(1e3 * t_port * args.procs / args.frames, 2)},
        "port_speed_over_reference": round(t_ref / t_port, 3),
        "max_param_diff_rel": diff,
        "python": sys.version.split()[0],
    }
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
