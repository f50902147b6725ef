"""The batched alignment hot path of one frame slab on one GPU.

match (K1, GPU) -> consensus (host, native) -> RANSAC (K2, GPU) -> affine
post-processing (host) -> warp (K3, GPU).  This is VideoAligner.align_images
(VA:57-158) after detection, with the three joblib stages (VA:117-123, 137-142, 150)
replaced by one batched launch each.  Frames and keypoints stay resident in HBM;
only survivor bitmasks (F x n_tpl/8 B), RANSAC point lists and 2x3 affines cross
PCIe.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch

from . import affines as _aff
from . import stages


@dataclass
class AlignConfig:
    """The reference's class constants that steer the hot path (VA:19-45)."""

    n_kp_global: int
    n_kp_global_min: int = 5            # N_KP_GLOBAL_MIN
    n_kp_frame_skip: int = 3            # N_KP_FRAME_SKIP
    ratio: float = 0.75                 # DESCRIPTOR_DISTANCE_RATIO_THRESH
    d_lo: float = 0.5                   # (d_1, d_2) hard-coded at VA:209
    d_hi: float = 2.0
    ransac_trials: int = 1000           # RANSAC_MAX_TRIALS
    ransac_threshold: float = 2.0       # RANSAC_RESIDUAL_THRESH
    ransac_min_samples: int = 2         # RANSAC_MIN_SAMPLES
    seed: int = 42                      # RANDOM_SEED
    spatial_rate: float = 1             # SPATIAL_DOWNSAMPLE_RATE
    frame_downsample_rate: int = 1      # max(1, frame_rate // FRAME_SAMPLE_RATE)
    # Extension (BASELINE configs 3-5): the skimage model class RANSAC fits.  The
    # reference always uses "euclidean" (EuclideanTransform, VA:311).
    ransac_model: str = "euclidean"     # "euclidean" | "affine" | "projective"
    # Opt-in (not the reference's matcher): BFMatcher norm, "l2" (the reference's
    # cv2.BFMatcher() default, VA:194) or "hamming" (NORM_HAMMING for binary descriptors).
    match_norm: str = "l2"

    @property
    def effective_frame_skip(self) -> int:
        """Frames with fewer points get NaN: N_KP_FRAME_SKIP, raised to min_samples + 1
        for the extension models (skimage needs min_samples < N, fit.py:798)."""
        if self.ransac_model == "euclidean":
            return self.n_kp_frame_skip
        return max(self.n_kp_frame_skip, {"affine": 3, "projective": 4}[self.ransac_model] + 1)


@dataclass
class SlabInputs:
    """Device-resident inputs of one slab.  Keypoints/descriptors are per SAMPLE frame
    (images[::frame_downsample_rate]); frames are the full uint16 stack to warp."""

    frames: torch.Tensor          # [F, H, W] (or [F, H, W, C]) uint16
    des_tpl: torch.Tensor         # [n_tpl, D] uint8
    kp_tpl: torch.Tensor          # [n_tpl, 2] float64
    des_q: torch.Tensor           # [P, D] uint8, CSR over sample frames
    kp_q: torch.Tensor            # [P, 2] float64
    q_off: torch.Tensor           # [S+1] int32 (device)
    q_off_host: np.ndarray        # same offsets on the host


@dataclass
class SlabResult:
    aligned: torch.Tensor
    affines: np.ndarray           # [S*rate, 2, 3] after interpolation (VA:143-144)
    euclidean: np.ndarray         # [S*rate, 3]
    skipped: List[int]
    interpolated: List[int]
    match: Optional[stages.MatchResult] = None
    consensus: Optional[stages.Consensus] = None
    ransac: Optional[stages.RansacResult] = None
    log_counts: Optional[np.ndarray] = None
    extras: dict = field(default_factory=dict)


def log_frame_counts(logger: logging.Logger, counts: np.ndarray, first_index: int = 0) -> None:
    """The per-frame debug lines of VA:215-221 / VA:125-126."""
    if not logger.isEnabledFor(logging.DEBUG):
        return
    for k, c in enumerate(counts):
        logger.debug(
            f"frame {first_index + k}:\n"
            f"\t{int(c[0])} unfiltered features identified\n"
            f"\t{int(c[1])} matches identified between frame and template\n"
            f"\t{int(c[2])} matches after feature-space ratio filter\n"
            f"\t{int(c[3])} matches after distance-based outlier rejection"
        )


def _nomark(name, ev=None):
    return None


def match_stage(inp: SlabInputs, cfg: AlignConfig, stream: Optional[int] = None) -> stages.MatchResult:
    """VA:194-214 for the slab."""
    return stages.match_frames(inp.des_tpl, inp.kp_tpl, inp.des_q, inp.kp_q, inp.q_off, inp.q_off_host,
                               ratio=cfg.ratio, d_lo=cfg.d_lo, d_hi=cfg.d_hi, norm=cfg.match_norm, stream=stream)


def _log_rates(logger: Optional[logging.Logger], votes: np.ndarray, n_frames: int) -> None:
    if logger is not None and logger.isEnabledFor(logging.INFO):
        rates = np.array(votes, dtype=np.int64) / n_frames
        logger.info(f"top n keypoints match rates: {rates}")


def _log_low_counts(logger: Optional[logging.Logger], ns: np.ndarray, cfg: AlignConfig, first_index: int = 0) -> None:
    """VA:279-283: frames whose consensus point list is shorter than N_KP_FRAME_SKIP."""
    if logger is None or not logger.isEnabledFor(logging.INFO):
        return
    for i in np.flatnonzero(ns < cfg.n_kp_frame_skip):
        logger.info(
            f"transform for frame {int(i) + first_index} not estimated due to low keypoint count: "
            f"({int(ns[i])}). Will be interpolated based on other frames instead"
        )


def consensus_stage(keep_bits_host: np.ndarray, n_tpl: int, n_frames: int, cfg: AlignConfig,
                    logger: Optional[logging.Logger] = None,
                    frames: Optional[Tuple[int, int]] = None) -> stages.Consensus:
    """VA:224-286 on the host from every frame's survivor bitmask.  With ``frames`` =
    (f_begin, f_end) the point lists are made for those frames only (pt_off starts at 0);
    the consensus and the per-frame log lines still cover every frame.  The pipelines use
    the device consensus (device_consensus / OverlappedSlabs) instead."""
    cons = stages.consensus(keep_bits_host, n_tpl, cfg.n_kp_global, cfg.n_kp_global_min, frames=frames)
    _log_rates(logger, cons.votes, n_frames)
    if logger is not None and logger.isEnabledFor(logging.INFO):
        if frames is None:
            ns = np.diff(cons.pt_off)
        else:  # every frame's point count = |consensus set & frame set|, from the bitmasks
            kb = np.ascontiguousarray(keep_bits_host).view(np.uint32)
            cbits = np.zeros(kb.shape[1], np.uint32)
            for k in np.asarray(cons.order, dtype=np.int64):
                cbits[k >> 5] |= np.uint32(1) << np.uint32(k & 31)
            ns = np.unpackbits((kb & cbits).view(np.uint8), axis=1).sum(axis=1)
        _log_low_counts(logger, ns, cfg)
    return cons


def choose_consensus(votes_host: np.ndarray, n_tpl: int, n_frames: int, cfg: AlignConfig,
                     logger: Optional[logging.Logger] = None,
                     pack_out: Optional[np.ndarray] = None) -> stages.ConsensusChoice:
    """VA:224-249 from the (merged) votes of every frame: Counter.most_common order,
    AlignmentError below N_KP_GLOBAL_MIN, the match-rate log line, set(consensus) order."""
    choice = stages.consensus_merge(votes_host, n_tpl, cfg.n_kp_global, cfg.n_kp_global_min, pack_out)
    _log_rates(logger, choice.votes, n_frames)
    return choice


def lookup_stage(match: stages.MatchResult, n_tpl: int, choice: stages.ConsensusChoice, pack_dev: torch.Tensor,
                 stream: Optional[int] = None) -> stages.Consensus:
    """VA:251-286 on the device: every frame's RANSAC point list (CSR, device)."""
    pt_off, pt_idx = stages.consensus_lookup(match.keep_bits, n_tpl, pack_dev, choice.nc, stream=stream)
    return stages.Consensus(choice.order, choice.votes, pt_off_dev=pt_off, pt_idx_dev=pt_idx)


def device_consensus(match: stages.MatchResult, n_tpl: int, n_frames: int, cfg: AlignConfig,
                     logger: Optional[logging.Logger] = None) -> stages.Consensus:
    """The whole consensus (VA:224-286) of one slab with the per-frame parts on the device
    (vote, lookup) and only the O(n_tpl) votes on the host (synchronous)."""
    votes = stages.consensus_vote(match.keep_bits, n_tpl)
    choice = choose_consensus(votes.cpu().numpy(), n_tpl, n_frames, cfg, logger)
    pack_dev = torch.from_numpy(choice.pack).to(match.keep_bits.device)
    cons = lookup_stage(match, n_tpl, choice, pack_dev)
    if logger is not None and logger.isEnabledFor(logging.INFO):
        _log_low_counts(logger, np.diff(cons.pt_off), cfg)
    return cons


def consensus_to_device(cons: stages.Consensus, dev) -> Tuple[torch.Tensor, torch.Tensor]:
    """Host consensus point lists (pt_off, pt_idx) as device tensors.  Stream-ordered
    copies from pinned staging (the caching host allocator keeps the staging alive until
    the copy has run): a pageable copy would block the host until the stream drains."""
    pt_off = torch.from_numpy(cons.pt_off).pin_memory().to(dev, non_blocking=True)
    pt_idx = torch.from_numpy(cons.pt_idx if cons.pt_idx.size else np.zeros(1, np.int32))
    return pt_off, pt_idx.pin_memory().to(dev, non_blocking=True)


def prepare_ransac(device, cfg: AlignConfig) -> None:
    """Hypothesis tables for every point count a device-consensus frame can have."""
    stages.ransac_prepare_range(device, cfg.ransac_model, max(cfg.effective_frame_skip, 3), cfg.n_kp_global,
                                cfg.ransac_trials, cfg.seed)


def _check_point_counts(cons: stages.Consensus, cfg: AlignConfig) -> None:
    """skimage raises when a frame is not skipped but has N <= min_samples (fit.py:798-799);
    only reachable when N_KP_FRAME_SKIP <= min_samples (the host then reads pt_off)."""
    ms = {"euclidean": cfg.ransac_min_samples, "affine": 3, "projective": 4}[cfg.ransac_model]
    skip = cfg.effective_frame_skip
    if skip > ms:
        return
    ns = np.diff(cons.pt_off)
    if ((ns >= skip) & (ns <= ms)).any():
        raise ValueError("`min_samples` must be in range (0, <number-of-samples>)")


def ransac_stage(match: stages.MatchResult, kp_tpl: torch.Tensor, cons: stages.Consensus,
                 cfg: AlignConfig, lists_dev: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 stream: Optional[int] = None, max_n: Optional[int] = None) -> stages.RansacResult:
    """VA:137-142: RANSAC of every frame's consensus points (src = the frame's matched
    keypoints, dst = template keypoints).  params [F, 2, 3] for the euclidean and
    affine models (model.params[:2], like VA:319), [F, 3, 3] for the projective one.
    Device point lists (device_consensus / lookup_stage) run with the tables of every
    count up to n_kp_global; host lists (consensus_stage) are uploaded first unless
    ``lists_dev`` holds them already."""
    if cfg.ransac_model == "euclidean" and cfg.ransac_min_samples != 2:
        # every path (host or device lists) fits EuclideanTransform's 2-point model
        raise ValueError("rigid RANSAC uses min_samples=2 (EuclideanTransform, VA:312)")
    dev = kp_tpl.device
    F, n_tpl = match.kp_ordered.shape[:2]
    src = match.kp_ordered.view(F * n_tpl, 2)
    if lists_dev is None and cons.pt_off_dev is not None:
        with stages.on_stream(dev, stream):  # pt_off is read after the lookup that wrote it
            _check_point_counts(cons, cfg)
        prepare_ransac(dev, cfg)
        rr = stages.ransac_lists(cfg.ransac_model, src, kp_tpl, cons.pt_off_dev, cons.pt_idx_dev, n_tpl,
                                 max_n=max_n if max_n is not None else max(len(cons.order), 1),
                                 trials=cfg.ransac_trials,
                                 residual_threshold=cfg.ransac_threshold, spatial_rate=cfg.spatial_rate,
                                 n_skip=cfg.effective_frame_skip, stream=stream)
    else:
        pt_off, pt_idx = lists_dev if lists_dev is not None else consensus_to_device(cons, dev)
        if cfg.ransac_model == "euclidean":
            return stages.ransac_rigid(src, kp_tpl, pt_off, cons.pt_off, pt_idx=pt_idx,
                                       src_frame_stride=n_tpl, trials=cfg.ransac_trials,
                                       residual_threshold=cfg.ransac_threshold, spatial_rate=cfg.spatial_rate,
                                       n_skip=cfg.n_kp_frame_skip, seed=cfg.seed, min_samples=cfg.ransac_min_samples)
        rr = stages.ransac_model(src, kp_tpl, pt_off, cons.pt_off, model=cfg.ransac_model,
                                 pt_idx=pt_idx, src_frame_stride=n_tpl, trials=cfg.ransac_trials,
                                 residual_threshold=cfg.ransac_threshold, spatial_rate=cfg.spatial_rate,
                                 n_skip=cfg.effective_frame_skip, seed=cfg.seed)
    if cfg.ransac_model == "affine":
        rr.params = rr.params[:, :2].contiguous()
    return rr


def postprocess_affines(params_host: np.ndarray, cfg: AlignConfig):
    """VA:143-145 on the host: NaN-pad, interpolate, Euclidean summary.  The
    reference's rotation-angle lerp (VA:409-437) assumes rigid matrices; the extension
    models interpolate their gaps entry-wise linearly instead.  Every frame with a model
    and no temporal downsampling (the common case) is one copy."""
    a = np.asarray(params_host)
    if int(cfg.frame_downsample_rate) == 1 and not _aff._nan_rows(a).any():
        affines = np.array(a, dtype=np.float64, copy=True)
        return affines, [], [], _aff.euclidean_transforms(affines)
    affines, skipped = _aff.process_affines(a, cfg.frame_downsample_rate)
    if cfg.ransac_model == "euclidean":
        affines, interpolated = _aff.interpolate_affines(affines)
    else:
        affines, interpolated = _aff.interpolate_linear(affines)
    return affines, skipped, interpolated, _aff.euclidean_transforms(affines)


def warp_frames(frames: torch.Tensor, maps: torch.Tensor, out: Optional[torch.Tensor] = None,
                stream: Optional[int] = None) -> torch.Tensor:
    """VA:150 on the device: warpAffine for [F, 2, 3] maps, warpPerspective for [F, 3, 3]."""
    if maps.shape[1:] == (3, 3):
        return stages.warp_perspective_u16(frames, maps, out=out, stream=stream)
    return stages.warp_affine_u16(frames, maps, out=out, stream=stream)


def warp_stage(frames: torch.Tensor, affines: np.ndarray, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    F = frames.shape[0]
    a = torch.from_numpy(np.ascontiguousarray(affines[:F], dtype=np.float64)).to(frames.device)
    return warp_frames(frames, a, out=out)


def align_slab(inp: SlabInputs, cfg: AlignConfig, logger: Optional[logging.Logger] = None,
               out: Optional[torch.Tensor] = None, keep_intermediates: bool = False) -> SlabResult:
    """Run the whole hot path for one slab on the slab's device."""
    logger = logger or logging.getLogger("VideoAligner")
    n_tpl = inp.des_tpl.shape[0]
    n_sample = inp.q_off.numel() - 1
    match = match_stage(inp, cfg)
    counts = match.counts.cpu().numpy() if logger.isEnabledFor(logging.DEBUG) else None
    if counts is not None:
        log_frame_counts(logger, counts)
    cons = device_consensus(match, n_tpl, n_sample, cfg, logger)
    rr = ransac_stage(match, inp.kp_tpl, cons, cfg)
    params = rr.params.cpu().numpy()
    affines, skipped, interpolated, eu = postprocess_affines(params, cfg)
    aligned = warp_stage(inp.frames, affines, out=out)
    return SlabResult(aligned, affines, eu, skipped, interpolated,
                      match if keep_intermediates else None, cons if keep_intermediates else None,
                      rr if keep_intermediates else None, counts)


def _d2h_async(t: torch.Tensor, copy: torch.cuda.Stream,
               produced: Optional[torch.cuda.Event] = None) -> Tuple[torch.Tensor, torch.cuda.Event]:
    """Device->host copy of ``t`` (produced on the current stream; ``produced``: an event
    already recorded after it) into pinned memory on the side stream ``copy``, so that the
    kernel stream does not stop for it; the event marks its end."""
    if produced is None:
        produced = torch.cuda.Event()
        produced.record()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    with torch.cuda.stream(copy):
        copy.wait_event(produced)
        t.record_stream(copy)
        h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(copy)
    return h, ev


def _h2d_async(arrays, dev, copy: torch.cuda.Stream):
    """Host->device copies (pinned staging) on the side stream ``copy``; the current
    stream waits for them.  Returns the device tensors."""
    with torch.cuda.stream(copy):
        outs = [torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev, non_blocking=True) for a in arrays]
        ev = torch.cuda.Event()
        ev.record(copy)
    cur = torch.cuda.current_stream(dev)
    cur.wait_event(ev)
    for o in outs:
        o.record_stream(cur)
    return outs


class _Slot:
    """Pinned host staging and transfer events of one slab in flight; slots are reused by
    later slabs once their slab is finished (every transfer through them has completed)."""

    def __init__(self):
        self.bufs = {}
        self.votes_ev = torch.cuda.Event()
        self.params_ev = torch.cuda.Event()

    def buf(self, name: str, numel: int, dtype: torch.dtype) -> torch.Tensor:
        b = self.bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype:
            b = torch.empty(max(numel, 1), dtype=dtype, pin_memory=True)
            self.bufs[name] = b
        return b[:numel]


@dataclass
class _SlabInFlight:
    """A slab on its way through the pipeline: matched (votes on their way to the host),
    then fitted (consensus lookup + RANSAC queued, parameters on their way to the host)."""

    inp: SlabInputs
    out: Optional[torch.Tensor]
    f0: int
    match: stages.MatchResult
    slot: _Slot
    n_votes: int                                   # elements of the (gathered) votes
    matched: Optional[torch.cuda.Event] = None     # end of match(k) + vote
    cons: Optional[stages.Consensus] = None
    rr: Optional[stages.RansacResult] = None
    aligned: Optional[torch.Tensor] = None
    fitted_ev: Optional[torch.cuda.Event] = None   # end of RANSAC(k) on the analysis stream
    n_bound: int = 0                               # elements of the gathered boundaries (sharded)


class OverlappedSlabs:
    """Streams slabs through the hot path as a software pipeline.

    submit(slab k) queues, in this device order,

        kernel stream:    [match(k) -> vote(k)] -> warp(k-1) -> [waits RANSAC(k)] -> warp(k) ...
        analysis stream:  [match(k) -> vote(k)] -> lookup(k) -> RANSAC(k)   (beside warp(k-1))

    with the parameter and map transfers on a side stream and the votes / consensus set in
    the analysis stream's own order (between the kernels that make and read them); the
    match + vote run on the analysis stream with
    ``match_beside`` (c2 / c3 / c4: the kernel stream then carries only the warps) and on
    the kernel stream ahead of the warp otherwise (c5: its 4 ms float match beside the
    1.4 ms warp starves it).  The consensus (VA:224-286) runs in three parts:
    the vote (per template count + first occurrence, VA:239) on the device right behind the
    match, the merge (Counter.most_common, set(consensus), VA:240-248) on the host from the
    O(n_tpl) votes, and the per-frame lookup (VA:274) on the device in front of RANSAC, so
    only the votes, the consensus set and the parameters cross PCIe.  RANSAC(k) shares the
    CUs with warp(k-1) (the warp is bound by HBM at the speed of a plain copy and leaves VALU
    slots free).  The warp of a slab reads its RANSAC parameters where RANSAC left them: with
    frame_downsample_rate == 1 the reference's post-processing (VA:143-145) hands a frame
    with a model its own parameters, so only frames without a model need the host (NaN-gap
    interpolation); the warp writes zeros for those and they are warped again, with the
    filled maps, once the host has them.  With frame_downsample_rate > 1 every full-rate
    frame's map comes from the host interpolation, and the warp of slab k waits for it.
    Every slab runs every stage and its results equal ``align_slab``'s.  (Measured and
    retired schedules -- depth 3, RANSAC behind the warp, a fixed CU slice for the
    analysis, a narrow RANSAC grid, the device-side merge in the pipeline, warp-first
    queueing -- are recorded in DESIGN 6b-6d.)

    submit returns the SlabResult of the previous submission (None for the first);
    flush() finishes the slab still in flight and returns its result.
    ``res.extras["done"]`` is an event after the slab's last warp; ``aligned`` is ready once
    it has passed (or after synchronize()).

    With ``counts`` (frames per rank) the slabs are one rank's share of a frame-sharded
    job (frame_downsample_rate 1): the votes [2, n_tpl] and each slab's parameter boundary
    (first / last frame with a model, kcmc_params_boundary) are all-gathered over ``group``
    in the same stream order on every rank, so a rank's host work per step is O(its own
    frames + world * n_tpl).  A rank's result holds its own frames (``extras["f0"]`` = the
    global index of the first): affines / euclidean of those frames, skipped and
    interpolated as global indices inside them.

        ov = OverlappedSlabs(device, cfg)
        results = [r for r in (ov.submit(inp) for inp in slabs) if r is not None] + ov.flush()
        ov.synchronize()
    """

    def __init__(self, device, cfg: AlignConfig, logger: Optional[logging.Logger] = None,
                 counts: Optional[List[int]] = None, group=None, match_beside: bool = False):
        self.match_beside = bool(match_beside)
        if counts is not None and len(counts) > 1 and cfg.frame_downsample_rate != 1:
            # the rank's first frame is counted in sample frames, the affines in full-rate
            # frames: the same restriction as distributed.align_sharded
            raise ValueError("the sharded path requires frame_downsample_rate == 1 "
                             "(frame_rate < 2*FRAME_SAMPLE_RATE)")
        self.dev = torch.device(device)
        self.cfg = cfg
        self.logger = logger
        self.counts = counts
        self.group = group
        self.stream = torch.cuda.Stream(self.dev)  # match (unless beside) and warps
        self.copy = torch.cuda.Stream(self.dev)    # vote / consensus / params / map transfers
        self.ana = torch.cuda.Stream(self.dev)     # [match], lookup and RANSAC beside the warp
        self._hs = self.stream.cuda_stream
        self._hc = self.copy.cuda_stream
        self._ha = self.ana.cuda_stream
        self._rank = 0
        self._world = 1
        self._f0 = 0
        self._nccl = False
        if self._sharded():
            import torch.distributed as dist

            self._rank = dist.get_rank(group)
            self._world = dist.get_world_size(group)
            self._f0 = sum(counts[: self._rank])
            self._nccl = dist.get_backend(group) == "nccl"
        self._slots: List[_Slot] = []
        # host seconds spent blocked in event waits / inside the all-gathers (the rest of a
        # submit is the host's own work; tools/host_scaling.py)
        self.stats = {"wait_s": 0.0, "gather_s": 0.0, "merge_s": 0.0, "post_s": 0.0}
        self._fitted: Optional[_SlabInFlight] = None   # RANSAC queued, warp pending
        self._tail: Optional[torch.cuda.Event] = None   # an event at the kernel stream's tail
        self._ana_tail: Optional[torch.cuda.Event] = None  # the same for the analysis stream

    def _at_tail(self, mark, *names) -> torch.cuda.Event:
        """One (timing) event at the kernel stream's current tail, shared by every wait,
        transfer and mark at this position: each event record is a marker packet, and the
        device spends ~10 us on every marker that sits between two kernels."""
        if self._tail is None:
            self._tail = torch.cuda.Event(enable_timing=True)
            self._tail.record(self.stream)
        for n in names:
            mark(n, self._tail)
        return self._tail

    def _queued(self) -> None:
        """Work was queued on the kernel stream: the tail event moves."""
        self._tail = None

    def _tail_on(self, stream: torch.cuda.Stream, mark, *names) -> torch.cuda.Event:
        """_at_tail for any of the pipeline's streams: the analysis stream's RANSAC end, the
        parameter transfer's dependency, the warp's wait and the next match's start mark
        share one marker packet (c3 trace: four markers between RANSAC and the next knn2
        cost ~20 us of idle device per step)."""
        if stream is self.stream:
            return self._at_tail(mark, *names)
        ev = self._ana_tail
        if ev is None:
            ev = self._ana_tail = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
        for n in names:
            mark(n, ev)
        return ev

    def _queued_on(self, stream: torch.cuda.Stream) -> None:
        if stream is self.stream:
            self._queued()
        else:
            self._ana_tail = None

    def _sharded(self) -> bool:
        return self.counts is not None and len(self.counts) > 1

    def _device_maps(self) -> bool:
        return int(self.cfg.frame_downsample_rate) == 1

    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        """All-gather of an equally sized tensor over the ranks, on the current stream:
        [world, *t.shape]."""
        import torch.distributed as dist

        t0 = time.perf_counter()
        out = torch.empty((self._world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if self._nccl:
            dist.all_gather_into_tensor(out, t, group=self.group)
        else:
            dist.all_gather(list(out.unbind(0)), t, group=self.group)
        self.stats["gather_s"] += time.perf_counter() - t0
        return out

    def _wait(self, ev: torch.cuda.Event) -> None:
        t0 = time.perf_counter()
        ev.synchronize()
        self.stats["wait_s"] += time.perf_counter() - t0

    def _d2h(self, host: torch.Tensor, src: torch.Tensor, after: torch.cuda.Event, done: torch.cuda.Event) -> None:
        """src (device) -> host (pinned) on the copy stream behind ``after``; ``done`` after it."""
        self.copy.wait_event(after)
        src.record_stream(self.copy)
        stages.memcpy_async(host.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), self._hc)
        done.record(self.copy)

    def _d2h_ana(self, host: torch.Tensor, src: torch.Tensor, done: torch.cuda.Event) -> None:
        """src (device) -> host (pinned) in the analysis stream's own order, ``done`` after it:
        the analysis chain's transfers sit between two of its own kernels, and a copy on the
        side stream costs the chain two cross-stream waits (tens of microseconds each on the
        device, c3 trace)."""
        stages.memcpy_async(host.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), self._ha)
        done.record(self.ana)
        self._queued_on(self.ana)

    def submit(self, inp: SlabInputs, out: Optional[torch.Tensor] = None,
               mark: Optional[Callable[[str, Optional[torch.cuda.Event]], None]] = None) -> Optional[SlabResult]:
        """``mark(name, event)``: stage marks m0/m1 (match + vote), w0/w1 (warp), r0/r1
        (lookup + RANSAC) with an event the pipeline recorded at that position."""
        mark = mark or _nomark
        self._wait_current()
        with torch.cuda.stream(self.stream):
            for t in (inp.frames, out):
                if t is not None:
                    t.record_stream(self.stream)
            fitted, self._fitted = self._fitted, None
            new = self._match(inp, out, mark)  # match(k): analysis stream (beside) or kernel stream
            if fitted is not None and self._device_maps():
                self._warp_device_maps(fitted, mark)  # warp(k-1)
            self._fitted = self._fit(new, mark)  # lookup + RANSAC(k) beside warp(k-1)
            return self._finish(fitted, mark) if fitted is not None else None

    def _wait_current(self) -> None:
        """Order the pipeline's streams after the caller's stream (the slab's inputs), but
        only when the caller's stream still has work queued: a cross-stream wait that is
        already satisfied still costs the device tens of microseconds.  The stream itself is
        asked (hipStreamQuery): recording a probe event on it every submit delayed the next
        match by ~11 us after the warp (`tools/gap_probe.py`: 41.5 -> 30.4 us)."""
        cur = torch.cuda.current_stream(self.dev)
        if cur == self.stream or cur.query():
            return
        ev = torch.cuda.Event()
        ev.record(cur)
        self.stream.wait_event(ev)
        if self.match_beside:  # the analysis stream reads the slab's keypoints
            self.ana.wait_event(ev)
            self._queued_on(self.ana)
        self._queued()

    def _match(self, inp: SlabInputs, out: Optional[torch.Tensor], mark) -> _SlabInFlight:
        """match(k) and its vote; the (gathered) votes to the host."""
        if self.match_beside:
            return self._match_beside(inp, out, mark)
        self._at_tail(mark, "m0")
        for t in (inp.des_tpl, inp.kp_tpl, inp.des_q, inp.kp_q, inp.q_off):
            t.record_stream(self.stream)
        n_tpl = inp.des_tpl.shape[0]
        match = match_stage(inp, self.cfg, stream=self._hs)
        votes = stages.consensus_vote(match.keep_bits, n_tpl, self._f0, stream=self._hs)
        self._queued()
        matched = self._at_tail(mark, "m1")
        if self._sharded():
            votes = self._gather(votes)  # the kernel stream waits for the collective
            self._queued()
        slot = self._slots.pop() if self._slots else _Slot()
        ready = self._at_tail(mark)
        self._d2h(slot.buf("votes", votes.numel(), torch.int64), votes, ready, slot.votes_ev)
        return _SlabInFlight(inp, out, self._f0, match, slot, votes.numel(), matched=matched)

    def _match_beside(self, inp: SlabInputs, out: Optional[torch.Tensor], mark) -> _SlabInFlight:
        """match(k) and its vote on the analysis stream (allocated there), behind the lookup +
        RANSAC of the previous slab; the (gathered) votes to the host."""
        n_tpl = inp.des_tpl.shape[0]
        with torch.cuda.stream(self.ana):
            # the match reads the slab's descriptors / keypoints on the analysis stream: keep
            # their memory from being reused by the caller's stream until it has
            for t in (inp.des_tpl, inp.kp_tpl, inp.des_q, inp.kp_q, inp.q_off):
                t.record_stream(self.ana)
            self._tail_on(self.ana, mark, "m0")  # usually the previous slab's RANSAC end
            match = match_stage(inp, self.cfg, stream=self._ha)
            votes = stages.consensus_vote(match.keep_bits, n_tpl, self._f0, stream=self._ha)
            self._queued_on(self.ana)
            matched = self._tail_on(self.ana, mark, "m1")
            if self._sharded():
                votes = self._gather(votes)  # the analysis stream waits for the collective
                self._queued_on(self.ana)
            slot = self._slots.pop() if self._slots else _Slot()
            self._d2h_ana(slot.buf("votes", votes.numel(), torch.int64), votes, slot.votes_ev)
        return _SlabInFlight(inp, out, self._f0, match, slot, votes.numel(), matched=matched)

    def _fit(self, p: _SlabInFlight, mark) -> _SlabInFlight:
        """The consensus merge (host) and the lookup + RANSAC (analysis stream) of a matched
        slab."""
        cfg = self.cfg
        n_tpl = p.inp.des_tpl.shape[0]
        n_local = p.inp.q_off.numel() - 1
        n_all = sum(self.counts) if self._sharded() else n_local
        self._wait(p.slot.votes_ev)
        votes = p.slot.buf("votes", p.n_votes, torch.int64).numpy().reshape(-1, 2, n_tpl)
        words = (n_tpl + 31) // 32
        pack_h = p.slot.buf("pack", cfg.n_kp_global + words, torch.int32)
        t0 = time.perf_counter()
        choice = choose_consensus(votes, n_tpl, n_all, cfg, self.logger if self._rank == 0 else None,
                                  pack_out=pack_h.numpy())
        self.stats["merge_s"] += time.perf_counter() - t0
        with torch.cuda.stream(self.ana):
            pack_dev = torch.empty(pack_h.numel(), dtype=torch.int32, device=self.dev)
            if not self.match_beside:  # the match ran on the kernel stream
                self.ana.wait_event(p.matched)
            # the consensus set goes up in the analysis stream's own order, right in front of
            # the lookup that reads it (no cross-stream wait on the device)
            stages.memcpy_async(pack_dev.data_ptr(), pack_h.data_ptr(), pack_h.numel() * 4, self._ha)
            self._queued_on(self.ana)
            for t in (p.match.kp_ordered, p.match.keep_bits, p.inp.kp_tpl):
                t.record_stream(self.ana)
            self._fit_device(p, choice, pack_dev, mark)
            for t in (p.rr.params, p.rr.inliers, p.rr.n_inliers, p.rr.best_trial):
                t.record_stream(self.stream)
        return p

    def _fit_device(self, p: _SlabInFlight, choice: stages.ConsensusChoice, pack_dev: torch.Tensor, mark) -> None:
        """Lookup + RANSAC of a slab whose consensus is known, on the analysis stream (the
        current stream here)."""
        n_tpl = p.inp.des_tpl.shape[0]
        st, hs = self.ana, self._ha
        self._tail_on(st, mark, "r0")
        p.cons = lookup_stage(p.match, n_tpl, choice, pack_dev, stream=hs)
        p.rr = ransac_stage(p.match, p.inp.kp_tpl, p.cons, self.cfg, stream=hs)
        self._queued_on(st)
        after = self._tail_on(st, mark, "r1")
        p.fitted_ev = after  # the warp reads the parameters where RANSAC left them
        params = p.rr.params
        # the parameters leave on the side stream: in the analysis stream their copy would sit
        # in front of the next slab's match (c3 trace: +26 us before knn2)
        d2h = (lambda host, src: self._d2h(host, src, after, p.slot.params_ev))
        if self._sharded():
            bound = self._gather(stages.params_boundary(params, stream=hs))
            self._queued_on(st)
            after = self._tail_on(st, _nomark)
            p.n_bound = bound.numel()
            d2h(p.slot.buf("bound", bound.numel(), torch.float64), bound)
        if logging_enabled(self.logger):
            # the point counts for VA:279-283's log lines travel with the parameters (the
            # lines are written in _finish): reading pt_off here would block the host on the
            # analysis stream and break the overlap
            d2h(p.slot.buf("pt_off", p.cons.pt_off_dev.numel(), torch.int32), p.cons.pt_off_dev)
        d2h(p.slot.buf("params", params.numel(), torch.float64), params)

    def _warp_device_maps(self, p: _SlabInFlight, mark) -> None:
        # RANSAC(k) ran beside warp(k-1) on the analysis stream: the host waits for it (it
        # has nothing else to do before it blocks on this step's votes) instead of queueing a
        # cross-stream wait, which leaves the device idle for tens of microseconds even when
        # RANSAC finished long before (round 5, same box: a device-side wait when RANSAC is
        # still running, c2 / c3 / c4 / c5 within noise, profiles/r05_j_device_wait_ab.txt)
        self._wait(p.fitted_ev)
        self._at_tail(mark, "w0")
        # one-call warp (plan + tiles) on the kernel stream: planning it on the analysis
        # stream behind RANSAC measured slower (profiles/r05_k_plan_beside_ab.txt)
        p.aligned = warp_frames(p.inp.frames, p.rr.params, out=p.out, stream=self._hs)
        self._queued()
        self._at_tail(mark, "w1")

    def _finish(self, p: _SlabInFlight, mark) -> SlabResult:
        """Host post-processing of slab p (VA:143-145) and the warps that need its maps."""
        self._wait(p.slot.params_ev)  # after RANSAC(k): its parameters are on the host
        n = p.inp.frames.shape[0]
        if logging_enabled(self.logger) and "pt_off" in p.slot.bufs:
            pt_off = p.slot.buf("pt_off", p.cons.pt_off_dev.numel(), torch.int32).numpy()
            _log_low_counts(self.logger, np.diff(pt_off), self.cfg, p.f0)
        shape = tuple(p.rr.params.shape)
        params = p.slot.buf("params", p.rr.params.numel(), torch.float64).numpy().reshape(shape)
        t0 = time.perf_counter()
        if self._sharded():
            from .distributed import neighbours

            E = int(np.prod(shape[1:]))
            bounds = p.slot.buf("bound", p.n_bound, torch.float64).numpy().reshape(self._world, 2 + 2 * E)
            prev, nxt = neighbours(bounds, self.counts, self._rank)
            local, skipped, interpolated = _aff.fill_gaps_slab(params, p.f0, prev, nxt,
                                                               lerp=self.cfg.ransac_model == "euclidean")
            affines, eu = local, _aff.euclidean_transforms(local)
        else:
            affines, skipped, interpolated, eu = postprocess_affines(params, self.cfg)
            local = np.asarray(affines[:n], dtype=np.float64)
        self.stats["post_s"] += time.perf_counter() - t0
        self._slots.append(p.slot)
        if self._device_maps():
            # frames without a model were warped to zeros: warp them with the filled maps
            redo = np.zeros(n, bool)
            sk = np.asarray(skipped, dtype=np.int64) - p.f0
            redo[sk[(sk >= 0) & (sk < n)]] = True
            for a, b in _runs(redo):
                (m,) = _h2d_async((local[a:b],), self.dev, self.copy)
                warp_frames(p.inp.frames[a:b], m, out=p.aligned[a:b], stream=self._hs)
                self._queued()
            aligned = p.aligned
        else:
            (m,) = _h2d_async((local,), self.dev, self.copy)
            self._queued()
            self._at_tail(mark, "w0")
            aligned = warp_frames(p.inp.frames, m, out=p.out, stream=self._hs)
            self._queued()
            self._at_tail(mark, "w1")
        done = self._at_tail(mark)
        res = SlabResult(aligned, affines, eu, skipped, interpolated, match=p.match, consensus=p.cons, ransac=p.rr)
        res.extras["done"] = done
        res.extras["f0"] = p.f0
        return res

    def flush(self, mark: Optional[Callable[[str, Optional[torch.cuda.Event]], None]] = None) -> List[SlabResult]:
        """Finish the slab still in flight; its result (an empty list when none is)."""
        mark = mark or _nomark
        out: List[SlabResult] = []
        with torch.cuda.stream(self.stream):
            fitted, self._fitted = self._fitted, None
            if fitted is not None:
                if self._device_maps():
                    self._warp_device_maps(fitted, mark)
                out.append(self._finish(fitted, mark))
        return out

    def synchronize(self) -> None:
        self.stream.synchronize()
        self.ana.synchronize()
        self.copy.synchronize()


def logging_enabled(logger: Optional[logging.Logger]) -> bool:
    return logger is not None and logger.isEnabledFor(logging.INFO)


def _runs(mask: np.ndarray):
    """Maximal runs [a, b) of True in a boolean vector."""
    if not mask.any():
        return []
    d = np.diff(np.concatenate(([0], mask.astype(np.int8), [0])))
    return list(zip(np.flatnonzero(d == 1).tolist(), np.flatnonzero(d == -1).tolist()))


def align_streamed(frames_host: torch.Tensor, inp: SlabInputs, cfg: AlignConfig, slab: int = 64,
                   out_host: Optional[torch.Tensor] = None, logger: Optional[logging.Logger] = None):
    """The whole hot path for a stack that lives in (pinned) host memory: the end-to-end
    use of align_images (VA:57-158) when the video does not stay on the device.

    Phase A runs match -> consensus -> RANSAC -> affine post-processing for every frame
    (only keypoints/descriptors are on the device: ``inp.frames`` is not used and may be
    an empty placeholder).  Phase B streams the frames through the warp in slabs of
    ``slab`` frames with three streams and double-buffered device slabs: host->device
    copy of slab k+1, warp of slab k and device->host copy of slab k-1 overlap, so the
    rate is bound by PCIe (both directions) rather than HBM.  Returns
    (out_host, SlabResult without the aligned tensor)."""
    dev = inp.des_tpl.device
    F = frames_host.shape[0]
    if out_host is None:
        out_host = torch.empty(frames_host.shape, dtype=frames_host.dtype, pin_memory=True)
    n_tpl = inp.des_tpl.shape[0]
    match = match_stage(inp, cfg)
    keep = match.keep_bits.cpu().numpy()
    cons = consensus_stage(keep, n_tpl, inp.q_off.numel() - 1, cfg, logger)
    rr = ransac_stage(match, inp.kp_tpl, cons, cfg)
    affines, skipped, interpolated, eu = postprocess_affines(rr.params.cpu().numpy(), cfg)
    maps = torch.from_numpy(np.ascontiguousarray(affines[:F], dtype=np.float64)).to(dev)

    shape = (slab,) + tuple(frames_host.shape[1:])
    bin_ = [torch.empty(shape, dtype=frames_host.dtype, device=dev) for _ in range(2)]
    bout = [torch.empty(shape, dtype=frames_host.dtype, device=dev) for _ in range(2)]
    s_in, s_cmp, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    cur = torch.cuda.current_stream(dev)
    for s in (s_in, s_cmp, s_out):
        s.wait_stream(cur)
    in_ready = [torch.cuda.Event() for _ in range(2)]
    in_free = [None, None]   # warp done reading bin_[b]
    out_free = [None, None]  # device->host copy done reading bout[b]
    for k, f0 in enumerate(range(0, F, slab)):
        b = k & 1
        n = min(slab, F - f0)
        with torch.cuda.stream(s_in):
            if in_free[b] is not None:
                s_in.wait_event(in_free[b])
            bin_[b][:n].copy_(frames_host[f0:f0 + n], non_blocking=True)
            in_ready[b].record(s_in)
        with torch.cuda.stream(s_cmp):
            s_cmp.wait_event(in_ready[b])
            if out_free[b] is not None:
                s_cmp.wait_event(out_free[b])
            warp_frames(bin_[b][:n], maps[f0:f0 + n], out=bout[b][:n])
            ev = torch.cuda.Event()
            ev.record(s_cmp)
            in_free[b] = ev
        with torch.cuda.stream(s_out):
            s_out.wait_event(in_free[b])
            out_host[f0:f0 + n].copy_(bout[b][:n], non_blocking=True)
            ev2 = torch.cuda.Event()
            ev2.record(s_out)
            out_free[b] = ev2
    for s in (s_in, s_cmp, s_out):
        cur.wait_stream(s)
    for t in bin_ + bout:
        t.record_stream(cur)
    return out_host, SlabResult(None, affines, eu, skipped, interpolated, match=match, consensus=cons, ransac=rr)


def downsample_u8(frames_u8: torch.Tensor, template_u8: torch.Tensor, frame_downsample_rate: int,
                  spatial_downsample_rate) -> Tuple[torch.Tensor, torch.Tensor]:
    """VideoAligner._downsample (VA:494-506) on the device: every rate-th frame and, only
    when the rate is not 1, cv2.pyrDown of the sample frames and the template
    (stages.pyr_down_u8) with the reference's dstsize = tuple(shape // spatial rate), which
    OpenCV reads as (width, height) -- so non-square frames fail its size assertion just
    as the reference does."""
    rate = int(frame_downsample_rate)
    if rate == 1:
        return frames_u8, template_u8
    H, W = frames_u8.shape[-2:]
    dsize = (int(H // spatial_downsample_rate), int(W // spatial_downsample_rate))
    return (stages.pyr_down_u8(frames_u8[::rate].contiguous(), dsize),
            stages.pyr_down_u8(template_u8.reshape(1, H, W).contiguous(), dsize))


def detect_slab(frames: torch.Tensor, cfg: AlignConfig, template_index: Optional[int] = None,
                template: Optional[torch.Tensor] = None, orb_params=None, percentile: float = 99.99):
    """The front end of align_images (VA:93-123) on the device for a uint16 stack:
    normalisation (f2: exact 99.99th percentile + max-scale) and the build's
    ORB-style detector (f1) on the template and on every sample frame.  Returns
    (SlabInputs for align_slab, brightest)."""
    if frames.dim() != 3:
        raise ValueError("detection needs a grayscale stack [F, H, W]")
    F = frames.shape[0]
    brightest = stages.brightest_px(frames, percentile)
    u8 = stages.max_scale_u8(frames, brightest)
    if template is None:
        ti = int(F * 0.5) if template_index is None else int(template_index)
        tpl_u8 = u8[ti:ti + 1]
    else:
        tpl_u8 = stages.max_scale_u8(template.reshape(1, *template.shape[-2:]).contiguous(), brightest)
    u8, tpl_u8 = downsample_u8(u8, tpl_u8, cfg.frame_downsample_rate, cfg.spatial_rate)
    kt = stages.detect_orb(tpl_u8, orb_params)
    kq = stages.detect_orb(u8, orb_params)
    n_t = int(kt.count.cpu()[0])
    kp_q, des_q, q_off, q_off_host = stages.keypoints_csr(kq)
    inp = SlabInputs(frames, kt.des[0, :n_t].contiguous(), kt.kp[0, :n_t].contiguous(), des_q, kp_q, q_off,
                     q_off_host)
    return inp, brightest


def align_frames(frames: torch.Tensor, cfg: AlignConfig, template_index: Optional[int] = None,
                 orb_params=None, out: Optional[torch.Tensor] = None,
                 logger: Optional[logging.Logger] = None) -> SlabResult:
    """align_images (VA:57-158) entirely on the device for a device-resident uint16 stack:
    normalisation, detection, matching, consensus (host, native), RANSAC, gap filling
    (host) and warp."""
    inp, brightest = detect_slab(frames, cfg, template_index, orb_params=orb_params)
    res = align_slab(inp, cfg, logger=logger, out=out)
    res.extras["brightest"] = brightest
    res.extras["n_template_keypoints"] = int(inp.des_tpl.shape[0])
    return res
