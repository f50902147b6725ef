"""Per-rank host work of the frame-sharded pipelined step against the world size, at a
fixed slab per rank (BASELINE config 3: 2500 frames of 512x512 per rank, affine RANSAC).

    python tools/host_scaling.py [--config c3] [--worlds 1,2,4,8] [--steps 20] [--frames F]

Every rank runs on cuda:0 with the gloo backend (a rehearsal: one GPU cannot host several
RCCL ranks), so the device is shared and the steps are world-times slower; what this
measures is each rank's HOST side per submit, split into
  * busy:   the host's own work (launches, the consensus merge, gap filling, Python),
  * wait:   blocked in event waits for the shared device,
  * gather: inside the all-gathers (gloo copies CUDA tensors through the host and the
            ranks wait for each other there; RCCL on a real node is stream-ordered),
with the consensus merge (O(world x n_tpl)) and the post-processing (O(frames per rank))
shown separately.  Before round 3 every rank recounted the vote and re-ran the gap
filling over all F_total frames, which grew with the world size."""
import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, args, out_path):
    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import bench
    from kcmc_amd import distributed as kdist, pipeline

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bc = bench.CONFIGS[args.config]
    F = args.frames or bc.frames_per_gpu
    inp, _ = bench.make_inputs(bc, F, rank, dev)
    if rank != 0:
        inp.des_tpl.zero_()
        inp.kp_tpl.zero_()
    kdist.broadcast_template(inp.des_tpl, inp.kp_tpl)
    out = torch.empty_like(inp.frames)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    ov = pipeline.OverlappedSlabs(dev, cfg, counts=[F] * world if world > 1 else None, match_beside=bc.match_beside)
    rows = []
    for s in range(args.steps + 3):
        st0 = dict(ov.stats)
        t0 = time.perf_counter()
        ov.submit(inp, out=out)
        wall = time.perf_counter() - t0
        if s >= 3:
            d = {k: ov.stats[k] - st0[k] for k in st0}
            rows.append({"wall": wall, "busy": wall - d["wait_s"] - d["gather_s"], "wait": d["wait_s"],
                         "gather": d["gather_s"], "merge": d["merge_s"], "post": d["post_s"]})
    ov.flush()
    ov.synchronize()
    med = {k: round(1e3 * float(np.median([r[k] for r in rows])), 4) for k in rows[0]}
    allm = [None] * world
    dist.all_gather_object(allm, med)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(allm, f)
    dist.destroy_process_group()


def host_only(args):
    """The host work of one rank per step, without the shared-device and gloo effects of
    the rehearsal: the slab's survivor bitmasks and RANSAC parameters come from the GPU
    once (BASELINE config 3 slab), then, for each world size W (F_total = W x F_local):
      round 3 (this tree): merge of W ranks' [2, n_tpl] votes (kcmc_consensus_merge) +
                           gap filling of the rank's own frames (affines.fill_gaps_slab);
      round 2 (before):    the vote + consensus over all F_total bitmasks
                           (kcmc_consensus_slice with the rank's frame range) + the global
                           post-processing of all F_total parameter sets.
    Each timed as the median of `--steps` repetitions."""
    import numpy as np
    import torch

    import bench
    from kcmc_amd import affines as aff, distributed as kdist, pipeline, stages

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bc = bench.CONFIGS[args.config]
    F = args.frames or bc.frames_per_gpu
    inp, _ = bench.make_inputs(bc, F, 0, dev)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    n_tpl = inp.des_tpl.shape[0]
    m = pipeline.match_stage(inp, cfg)
    keep = m.keep_bits.cpu().numpy()
    cons = pipeline.device_consensus(m, n_tpl, F, cfg)
    params = pipeline.ransac_stage(m, inp.kp_tpl, cons, cfg).params.cpu().numpy()
    params[F // 3:F // 3 + 7] = np.nan  # a gap, so the gap filling has work to do
    votes1 = stages.consensus_vote_host(keep, n_tpl)

    def med(fn):
        ts = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(1e3 * float(np.median(ts)), 4)

    res = {}
    for w in [int(x) for x in args.worlds.split(",")]:
        votes = np.stack([votes1] * w)
        keep_all = np.concatenate([keep] * w)
        params_all = np.concatenate([params] * w)
        bounds = np.tile(np.concatenate(([0, F - 1], params[0].ravel(), params[-1].ravel())), (w, 1))
        counts = [F] * w
        r = w // 2  # a middle rank

        def new_step():
            pipeline.choose_consensus(votes, n_tpl, F * w, cfg)
            prev, nxt = kdist.neighbours(bounds, counts, r)
            loc, _, _ = aff.fill_gaps_slab(params, r * F, prev, nxt, lerp=cfg.ransac_model == "euclidean")
            aff.euclidean_transforms(loc)

        def old_step():
            pipeline.consensus_stage(keep_all, n_tpl, F * w, cfg, frames=(r * F, (r + 1) * F))
            pipeline.postprocess_affines(params_all, cfg)

        res[w] = {"f_total": F * w, "round3_host_ms": med(new_step), "round2_host_ms": med(old_step),
                  "merge_ms": med(lambda: pipeline.choose_consensus(votes, n_tpl, F * w, cfg)),
                  "fill_gaps_ms": med(lambda: aff.fill_gaps_slab(params, r * F, *kdist.neighbours(bounds, counts, r),
                                                                 lerp=cfg.ransac_model == "euclidean"))}
        print(f"world {w} (F_total {F * w}): round-3 host work {res[w]['round3_host_ms']:.3f} ms "
              f"(merge {res[w]['merge_ms']:.3f}, gap filling {res[w]['fill_gaps_ms']:.3f}); "
              f"round-2 host work {res[w]['round2_host_ms']:.3f} ms", flush=True)
    out = {"mode": "host-only", "config": args.config, "frames_per_rank": F, "worlds": res,
           "note": "per-rank host work per step that depends on the job size; round 2 recounted the vote and "
                   "re-ran the gap filling over all F_total frames on every rank"}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


def main():
    import numpy as np
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--out", default="gpurun_out/host_scaling.json")
    ap.add_argument("--rehearsal", action="store_true",
                    help="spawn `world` gloo ranks on cuda:0 and time whole submits (default: --host-only timing)")
    args = ap.parse_args()
    if not args.rehearsal:
        return host_only(args)
    res = {}
    for w in [int(x) for x in args.worlds.split(",")]:
        path = args.out + f".w{w}.tmp"
        mp.spawn(_rank, args=(w, _free_port(), args, path), nprocs=w, join=True)
        per_rank = json.load(open(path))
        os.remove(path)
        res[w] = {"per_rank_median_ms": per_rank,
                  "busy_ms_max_over_ranks": max(r["busy"] for r in per_rank),
                  "merge_ms_max": max(r["merge"] for r in per_rank),
                  "post_ms_max": max(r["post"] for r in per_rank)}
        print(f"world {w}: host busy per submit (max over ranks) {res[w]['busy_ms_max_over_ranks']:.3f} ms, "
              f"merge {res[w]['merge_ms_max']:.3f} ms, post-processing {res[w]['post_ms_max']:.3f} ms", flush=True)
    frames = args.frames or 2500
    out = {"config": args.config, "frames_per_rank": frames,
           "f_total": {w: w * frames for w in res}, "worlds": res,
           "note": "all ranks on cuda:0 with gloo (rehearsal); busy = submit wall - event waits - all-gather time"}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({w: res[w]["busy_ms_max_over_ranks"] for w in res}))
    del np


if __name__ == "__main__":
    main()
