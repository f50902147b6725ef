"""Frame-sharded hot path over several GPUs (one process per GPU, torch.distributed).

Frames are independent in every per-frame stage, so each rank owns a contiguous slab
of frames and runs K1/K2/K3 on it locally.  The reference has exactly two cross-frame
steps, and only those exchange data (RCCL over xGMI with the "nccl" backend), each
O(n_tpl) or O(1) per rank -- never O(frames):

  1. the keypoint consensus vote (VA:224-286): each rank reduces its own frames' survivor
     bitmasks on the device to per-template votes (count + first occurrence,
     kcmc_consensus_vote), the [2, n_tpl] votes are all-gathered (world x 16 x n_tpl B:
     8 x 500 x 16 = 64 KB at config 3), every rank merges them on the host into the same
     Counter.most_common consensus (kcmc_consensus_merge) and looks up the RANSAC point
     lists of its own frames on the device (kcmc_consensus_lookup);
  2. the NaN-gap interpolation (VA:347-407) only needs, across ranks, the nearest frames
     with a model on either side of a slab: each rank's first / last such frame and its
     parameters are all-gathered ((2 + 2E) doubles per rank), and each rank fills the gaps
     of its own frames (affines.fill_gaps_slab).
The template descriptors/keypoints are broadcast once from rank 0 (VA:117-123 pickles
them to every worker).  Global frame order is rank-major: rank r owns frames
[sum_{q<r} F_q, ... + F_r).  A rank's results cover its own frames and equal the rows
[f0, f0 + F_r) of a single-device run (gather_results assembles the global arrays).

The compute stages are pluggable (``SlabStages``) so the exchange logic can be tested
on CPU ranks with the gloo backend; the product default runs the HIP kernels.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import affines as _aff
from . import pipeline as _pl
from . import stages


@dataclass
class SlabStages:
    """Per-rank compute:
    match(inp, cfg) -> (keep_bits [F, W] i32 tensor, kp_ordered [F, n_tpl, 2] f64 tensor);
    vote(keep_bits, n_tpl, frame_base) -> [2, n_tpl] i64 tensor (kcmc_consensus_vote);
    lookup(keep_bits, n_tpl, choice) -> stages.Consensus with the point lists of these frames;
    ransac(kp_ordered, kp_tpl, cons, cfg) -> params [F, 2, 3] / [F, 3, 3] f64 tensor;
    boundary(params) -> [2 + 2E] f64 tensor (kcmc_params_boundary);
    warp(frames, affines_host [F, ...]) -> aligned tensor;
    warp_params(frames, params) -> aligned tensor: the warp with ransac's own parameters
    where they lie (a frame without a model -- NaN parameters -- comes out as zeros), or
    None when the stages have no such warp."""

    match: Callable
    vote: Callable
    lookup: Callable
    ransac: Callable
    boundary: Callable
    warp: Callable
    warp_params: Optional[Callable] = None


def _hip_match(inp: _pl.SlabInputs, cfg: _pl.AlignConfig):
    m = _pl.match_stage(inp, cfg)
    return m.keep_bits, m.kp_ordered


def _hip_vote(keep_bits: torch.Tensor, n_tpl: int, frame_base: int) -> torch.Tensor:
    return stages.consensus_vote(keep_bits, n_tpl, frame_base)


def _hip_lookup(keep_bits: torch.Tensor, n_tpl: int, choice: stages.ConsensusChoice) -> stages.Consensus:
    pack_dev = torch.from_numpy(choice.pack).to(keep_bits.device)
    pt_off, pt_idx = stages.consensus_lookup(keep_bits, n_tpl, pack_dev, choice.nc)
    return stages.Consensus(choice.order, choice.votes, pt_off_dev=pt_off, pt_idx_dev=pt_idx)


def _hip_ransac(kp_ordered: torch.Tensor, kp_tpl: torch.Tensor, cons: stages.Consensus,
                cfg: _pl.AlignConfig) -> torch.Tensor:
    m = stages.MatchResult(None, None, kp_ordered, None, None)
    return _pl.ransac_stage(m, kp_tpl, cons, cfg).params


def _hip_warp(frames: torch.Tensor, affines: np.ndarray) -> torch.Tensor:
    return _pl.warp_stage(frames, affines)


def _hip_warp_params(frames: torch.Tensor, params: torch.Tensor) -> torch.Tensor:
    return _pl.warp_frames(frames, params)


HIP_STAGES = SlabStages(_hip_match, _hip_vote, _hip_lookup, _hip_ransac, stages.params_boundary, _hip_warp,
                        _hip_warp_params)


def _all_gather_rows(t: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """All-gather a [F_r, ...] tensor whose first dimension differs per rank."""
    world = dist.get_world_size(group)
    fmax = max(counts)
    pad = torch.zeros((fmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([outs[r][: counts[r]] for r in range(world)], 0)


def all_gather_equal(t: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather of an equally sized tensor: [world, *t.shape]."""
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if t.device.type == "cuda" and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    else:
        dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group)
    return out


def neighbours(bounds: np.ndarray, counts: List[int], rank: int):
    """From the all-gathered params boundaries [world, 2 + 2E]: (global index, model) of
    the last frame with a model before this rank's slab and of the first one after it
    (None where no rank has one)."""
    E = (bounds.shape[1] - 2) // 2
    starts = np.concatenate(([0], np.cumsum(counts)))
    prev = nxt = None
    for q in range(rank - 1, -1, -1):
        if bounds[q, 1] >= 0:
            prev = (int(starts[q] + bounds[q, 1]), bounds[q, 2 + E:2 + 2 * E].copy())
            break
    for q in range(rank + 1, len(counts)):
        if bounds[q, 0] >= 0:
            nxt = (int(starts[q] + bounds[q, 0]), bounds[q, 2:2 + E].copy())
            break
    return prev, nxt


def broadcast_template(des_tpl: torch.Tensor, kp_tpl: torch.Tensor, group=None, src: int = 0):
    dist.broadcast(des_tpl, src=src, group=group)
    dist.broadcast(kp_tpl, src=src, group=group)
    return des_tpl, kp_tpl


def frame_counts(n_local: int, device: torch.device, group=None) -> List[int]:
    world = dist.get_world_size(group)
    t = torch.tensor([n_local], dtype=torch.int64, device=device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [int(o.item()) for o in outs]


def align_sharded(inp: _pl.SlabInputs, cfg: _pl.AlignConfig, group=None, impl: SlabStages = HIP_STAGES,
                  logger: Optional[logging.Logger] = None, counts: Optional[List[int]] = None) -> _pl.SlabResult:
    """One rank's share of align_images: this rank's aligned frames, affines, Euclidean
    transforms (rows of its frames), skipped and interpolated frames (global indices inside
    its slab); ``extras["f0"]`` = the global index of its first frame.  Host work and
    exchanged bytes per rank do not grow with the number of frames on the other ranks."""
    if cfg.frame_downsample_rate != 1:
        raise ValueError("the sharded path requires frame_downsample_rate == 1 (frame_rate < 2*FRAME_SAMPLE_RATE)")
    rank = dist.get_rank(group)
    dev = inp.kp_tpl.device
    n_local = inp.q_off.numel() - 1
    if counts is None:
        counts = frame_counts(n_local, dev, group)
    f0 = sum(counts[:rank])
    n_tpl = inp.des_tpl.shape[0]
    # K1 + the vote on the local slab, then exchange the votes (exchange step 1)
    keep_bits, kp_ordered = impl.match(inp, cfg)
    votes = all_gather_equal(impl.vote(keep_bits, n_tpl, f0), group).cpu().numpy()
    choice = _pl.choose_consensus(votes, n_tpl, sum(counts), cfg, logger if rank == 0 else None)
    cons = impl.lookup(keep_bits, n_tpl, choice)
    params = impl.ransac(kp_ordered, inp.kp_tpl, cons, cfg)
    # exchange the slab boundaries (exchange step 2), then fill this slab's gaps
    bounds = all_gather_equal(impl.boundary(params), group).cpu().numpy()
    prev, nxt = neighbours(bounds, counts, rank)
    local, skipped, interpolated = _aff.fill_gaps_slab(params.cpu().numpy(), f0, prev, nxt,
                                                       lerp=cfg.ransac_model == "euclidean")
    aligned = impl.warp(inp.frames, local)
    res = _pl.SlabResult(aligned, local, _aff.euclidean_transforms(local), skipped, interpolated, consensus=cons)
    res.extras["f0"] = f0
    return res


def gather_results(res: _pl.SlabResult, counts: List[int], group=None):
    """The global (all-frame) affines, Euclidean transforms, skipped and interpolated lists
    of a sharded job from every rank's SlabResult (O(total frames) per rank: for callers
    that want the single-device return values of align_images, not for the step loop)."""
    dev = torch.device("cpu") if dist.get_backend(group) != "nccl" else torch.device("cuda", torch.cuda.current_device())
    aff = _all_gather_rows(torch.from_numpy(np.ascontiguousarray(res.affines)).to(dev), counts, group).cpu().numpy()
    eu = _all_gather_rows(torch.from_numpy(np.ascontiguousarray(res.euclidean)).to(dev), counts, group).cpu().numpy()
    lists = [None] * dist.get_world_size(group)
    dist.all_gather_object(lists, (list(res.skipped), list(res.interpolated)), group=group)
    skipped = [i for s, _ in lists for i in s]
    interpolated = [i for _, it in lists for i in it]
    return aff, eu, skipped, interpolated


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's environment (RANK,
    WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, local_rank)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local
