"""Benchmark of the alignment hot path on BASELINE.json config[1]:
1080p grayscale uint16, 2000 frames per GPU, ORB-like keypoints (500 per template,
32-byte descriptors, ~550 per frame), rigid RANSAC (1000 trials), n_kp_global = 100.

One step = one pass of the hot path over the whole batch with inputs resident in HBM:
K1 match (GPU) -> survivor bitmasks to host -> consensus (host, native) -> K2 RANSAC
(GPU) -> affine post-processing (host) -> K3 warp of every uint16 frame (GPU).
Detection is not part of the path (no detector exists in this image; keypoints are
synthetic, see kcmc_amd/synthetic.py).

Steps are issued through pipeline.OverlappedSlabs: match/consensus/RANSAC of step k+1
run (analysis stream + host) while step k's frames are warped (warp stream); every step
still runs every stage.  --serial runs the steps strictly one after another.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  value = frames aligned by all ranks / max-over-ranks
wall time of the K timed steps.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import kcmc_amd  # noqa: E402,F401
from kcmc_amd import distributed as kdist  # noqa: E402
from kcmc_amd import pipeline, stages, synthetic  # noqa: E402

METRIC = "aligned frames/sec (whole node) at 1080p; RANSAC hypotheses scored/sec/GPU"
H, W = 1080, 1920
N_TPL, D = 500, 32
N_KP_GLOBAL = 100
TRIALS = 1000
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_inputs(frames_per_gpu: int, rank: int, dev: torch.device):
    ks = synthetic.make_keypoints(frames_per_gpu, N_TPL, D, (H, W), seed=3, frame_seed=rank)
    base = synthetic.make_texture((H, W), seed=0)
    base_t = torch.from_numpy(base).to(dev)
    src = base_t.expand(frames_per_gpu, H, W).contiguous()
    # jittered video: each frame is the base texture seen through the inverse of its
    # ground-truth frame->template map (generated once, outside the timed region)
    frames = stages.warp_affine_u16(src, torch.from_numpy(ks.gt).to(dev), inverse_map=True)
    del src
    inp = pipeline.SlabInputs(
        frames=frames,
        des_tpl=torch.from_numpy(ks.des_tpl).to(dev),
        kp_tpl=torch.from_numpy(ks.kp_tpl).to(dev),
        des_q=torch.from_numpy(ks.des_q).to(dev),
        kp_q=torch.from_numpy(ks.kp_q).to(dev),
        q_off=torch.from_numpy(ks.q_off).to(dev),
        q_off_host=ks.q_off,
    )
    torch.cuda.synchronize(dev)
    return inp, ks


class StageTimer:
    """HIP events on the stream the kernels run on (torch's current stream)."""

    def __init__(self):
        self.ev = {}

    def mark(self, name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.setdefault(name, []).append(e)

    def elapsed(self, a, b):
        return [x.elapsed_time(y) for x, y in zip(self.ev[a], self.ev[b])]


def run_step(inp, cfg, out, timer=None, world=1, counts=None):
    """One pass of the hot path (single GPU or this rank's share of a sharded run)."""
    n_tpl = inp.des_tpl.shape[0]
    if timer:
        timer.mark("m0")
    m = pipeline.match_stage(inp, cfg)
    if timer:
        timer.mark("m1")
    if world > 1:
        keep_all = kdist._all_gather_rows(m.keep_bits, counts).cpu().numpy()
        n_all = sum(counts)
    else:
        keep_all = m.keep_bits.cpu().numpy()
        n_all = keep_all.shape[0]
    cons = pipeline.consensus_stage(keep_all, n_tpl, n_all, cfg)
    if world > 1:
        rank = torch.distributed.get_rank()
        f0, nl = sum(counts[:rank]), counts[rank]
        po = cons.pt_off
        lo, hi = int(po[f0]), int(po[f0 + nl])
        cons = stages.Consensus(cons.order, cons.votes, (po[f0:f0 + nl + 1] - lo).astype(np.int32),
                                cons.pt_idx[lo:hi])
    if timer:
        timer.mark("r0")
    rr = pipeline.ransac_stage(m, inp.kp_tpl, cons, cfg)
    if timer:
        timer.mark("r1")
    if world > 1:
        params = kdist._all_gather_rows(rr.params, counts).cpu().numpy()
    else:
        params = rr.params.cpu().numpy()
    affines, skipped, interp, eu = pipeline.postprocess_affines(params, cfg)
    if world > 1:
        rank = torch.distributed.get_rank()
        f0 = sum(counts[:rank])
        affines = affines[f0:f0 + counts[rank]]
    a_dev = torch.from_numpy(np.ascontiguousarray(affines[: inp.frames.shape[0]])).to(inp.frames.device)
    if timer:
        timer.mark("w0")
    stages.warp_affine_u16(inp.frames, a_dev, out=out)
    if timer:
        timer.mark("w1")
    return cons, rr


def cpu_baseline(ks, n_sample: int):
    """The oracle restatement of the reference CPU path on a bounded sample (1 thread):
    C knnMatch + the reference's numpy filters, CPython consensus, the numpy/LAPACK
    restatement of skimage 0.18.3 ransac (per-trial SVD, like the reference), C warpAffine."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # cpu_baseline leg: the oracle is what is timed here
    from threadpoolctl import threadpool_limits

    base = synthetic.make_texture((H, W), seed=0)
    with threadpool_limits(1):
        t0 = time.perf_counter()
        sets, kqs = [], []
        for f in range(n_sample):
            a, b = ks.q_off[f], ks.q_off[f + 1]
            idx, dist = oracle.knn2_l2u8(ks.des_tpl, ks.des_q[a:b])
            s, kq, _ = oracle.filter_matches(idx, dist, ks.kp_tpl, ks.kp_q[a:b])
            sets.append(s)
            kqs.append(kq)
        t1 = time.perf_counter()
        cons, _, _ = oracle.consensus(sets, N_KP_GLOBAL)
        lists = oracle.lookup(cons, sets)
        t2 = time.perf_counter()
        affs = []
        for f in range(n_sample):
            L = lists[f]
            if len(L) < 3:
                affs.append(np.full((2, 3), np.nan))
                continue
            p, _ = oracle.ransac_rigid_skimage(kqs[f][L], ks.kp_tpl[L])
            affs.append(p)
        t3 = time.perf_counter()
        for f in range(n_sample):
            oracle.warp_affine_u16(base, affs[f])
        t4 = time.perf_counter()
    total = t4 - t0
    return {
        "value": n_sample / total,
        "unit": "aligned frames/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{n_sample} frames of config[1] (1080p u16, n_tpl=500, D=32, n_kp_global=100), 1 thread: "
                   f"match {1e3 * (t1 - t0) / n_sample:.1f} ms/frame (C oracle knnMatch + reference numpy filters), "
                   f"consensus {1e3 * (t2 - t1):.1f} ms (CPython set/Counter), "
                   f"RANSAC {1e3 * (t3 - t2) / n_sample:.1f} ms/frame (numpy/LAPACK restatement of skimage 0.18.3, "
                   f"1000 trials), warp {1e3 * (t4 - t3) / n_sample:.1f} ms/frame (C oracle warpAffine)"),
        "seconds": total,
    }


def load_traffic():
    """HBM bytes per warp launch from the committed rocprofv3 PMC pass, if present."""
    p = os.path.join(REPO, "profiles", "warp_pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), d
    except (OSError, ValueError):
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=2000, help="frames per GPU (config[1]: 2000)")
    ap.add_argument("--cpu-sample", type=int, default=240, help="frames in the CPU-baseline sample (0: skip)")
    ap.add_argument("--serial", action="store_true",
                    help="run steps back to back on one stream (no warp/analysis overlap between steps)")
    args = ap.parse_args()

    rank, world, local = kdist.init_from_env("nccl")
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    t_setup = time.perf_counter()
    inp, ks = make_inputs(args.frames, rank, dev)
    out = torch.empty_like(inp.frames)
    cfg = pipeline.AlignConfig(n_kp_global=N_KP_GLOBAL)
    counts = [args.frames] * world
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s; {args.frames} frames {H}x{W} on {dev}")

    ov = None if args.serial else pipeline.OverlappedSlabs(dev, cfg, counts=counts if world > 1 else None)

    def step(timer):
        if ov is None:
            return run_step(inp, cfg, out, timer, world, counts)
        res, _ = ov.submit(inp, out=out, mark=timer.mark if timer else None)
        return res.consensus, res.ransac

    for _ in range(args.warmup):
        step(None)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    timer = StageTimer()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cons, rr = step(timer)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = 1e3 * elapsed / args.steps
    total_frames = args.frames * world
    fps = total_frames * args.steps / elapsed
    warp_ms = float(np.mean(timer.elapsed("w0", "w1")))
    match_ms = float(np.mean(timer.elapsed("m0", "m1")))
    ransac_ms = float(np.mean(timer.elapsed("r0", "r1")))
    n_pts = np.diff(cons.pt_off)
    if len(n_pts) > args.frames:  # overlapped multi-rank steps return the global consensus
        n_pts = n_pts[rank * args.frames:(rank + 1) * args.frames]
    n_ransac = int((n_pts >= cfg.n_kp_frame_skip).sum())
    warp_bytes = 2 * inp.frames.numel() * inp.frames.element_size()  # read + write, algorithmic
    achieved = warp_bytes / (warp_ms * 1e-3) / 1e9
    traffic, _ = load_traffic()
    stage_ms = {"match": round(match_ms, 3), "ransac": round(ransac_ms, 3), "warp": round(warp_ms, 3)}
    if ov is None:
        stage_ms["host_and_transfers"] = round(ms_step - match_ms - ransac_ms - warp_ms, 3)
    else:  # step k+1's match/consensus/RANSAC/post-processing overlap step k's warp
        stage_ms["schedule"] = "overlapped: analysis stream (match, RANSAC) + warp stream"
        stage_ms["step_minus_warp"] = round(ms_step - warp_ms, 3)
    result = {
        "metric": METRIC,
        "value": round(fps, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16 frames; i8 MFMA match, f64 RANSAC, f32 warp weights",
        "data": "synthetic (seeded jittered 1080p texture + ORB-shaped keypoints; no detector in image)",
        "config": {
            "workload": "BASELINE config[1]: 1080p grayscale u16, 2000 frames per GPU, ORB-like keypoints "
                        "(n_tpl=500, D=32 B, ~550/frame), rigid RANSAC 1000 trials, n_kp_global=100",
            "frames_per_gpu": args.frames, "height": H, "width": W, "n_tpl": N_TPL, "descriptor_bytes": D,
            "n_kp_global": N_KP_GLOBAL, "ransac_trials": TRIALS, "parallelism": f"frame-sharded x{world}",
        },
        "ransac_hypotheses_per_s_per_gpu": round(n_ransac * TRIALS / (ransac_ms * 1e-3), 1),
        "ransac_mean_points": round(float(n_pts.mean()), 2),
        "stage_ms": stage_ms,
        "roofline": {
            "kernel": "warp_affine_u16_kernel<1>",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": warp_bytes,
            "avg_launch_ms": round(warp_ms, 4),
        },
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        result["cpu_baseline"] = cpu_baseline(ks, args.cpu_sample)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
