"""Single-process alignment over several GPUs: the drop-in ``VideoAligner``'s path across
every visible device.

The reference spreads each of its three per-frame stages over every core of the machine
(``N_JOBS_PARALLEL = cpu_count()``, VA:21; ``_parallelize``, VA:460-471).  Its MI355X
equivalent splits the sample frames into one contiguous slab per device entry (SURVEY
8(e), the single-process form; ``distributed.align_sharded`` is the one-process-per-GPU
form) and keeps every cross-frame step on the host exactly once:

  1. per slab, queued on every device before the host waits for any: K1 match + the
     consensus vote of its frames (per template count + first occurrence with the slab's
     GLOBAL first sample index, kcmc_consensus_vote), the votes copied to the host;
  2. host: the votes of every slab merged ONCE (Counter.most_common + set(consensus) order,
     VA:224-249, kcmc_consensus_merge) -- the same merge a one-device run makes;
  3. per slab, queued on every device: the consensus lookup (VA:251-286) + K2 RANSAC, and
     without temporal downsampling the K3 warp right behind it with the parameters where
     RANSAC left them (a frame with a model keeps its own parameters through step 4);
  4. host: the parameters of every slab concatenated in frame order and post-processed once
     (NaN padding for temporal downsampling, gap interpolation across slab boundaries,
     VA:143-145), while the warps of step 3 run;
  5. per slab: K3 warp of its full-rate frames with its rows of the global maps (after a
     step-3 warp: only the frames without a model, which it left at zero).
Every per-frame stage is independent of the other frames, so the result equals
``pipeline.align_slab`` over the whole stack bit for bit (tests/test_gpu_multidevice.py
runs two slabs on one GPU against one slab).  A device may appear more than once in the
device list (two slabs on one GPU: the rehearsal of the split on a one-GPU box).

The compute stages are pluggable (``distributed.SlabStages``: match, vote, lookup,
ransac, warp) so the split / merge / post-processing logic runs in CPU tests with
stand-ins; the product default is the HIP stages.
"""
from __future__ import annotations

import contextlib
import logging
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import pipeline as _pl
from . import stages


@dataclass
class SlabRange:
    """One slab of a split: sample frames [s0, s1) (the frames keypoints belong to) and
    the full-rate frames [f0, f1) it warps (rate = frame_downsample_rate)."""

    s0: int
    s1: int
    f0: int
    f1: int


def split_frames(n_frames: int, rate: int, parts: int) -> List[SlabRange]:
    """Contiguous, balanced slabs of a stack of ``n_frames`` full-rate frames whose sample
    frames are images[::rate] (ceil(n_frames / rate) of them, VA:494-499).  Slab k's
    full-rate frames are the ones its sample frames stand for (f = s * rate ...
    s * rate + rate - 1), so the temporal NaN padding of VA:338-344 never straddles two
    slabs.  Empty slabs (more parts than sample frames) are dropped."""
    if n_frames < 0 or rate < 1 or parts < 1:
        raise ValueError("split_frames: need n_frames >= 0, rate >= 1, parts >= 1")
    n_sample = -(-n_frames // rate)
    out = []
    for chunk in np.array_split(np.arange(n_sample), parts):
        if chunk.size == 0:
            continue
        s0, s1 = int(chunk[0]), int(chunk[-1]) + 1
        out.append(SlabRange(s0, s1, s0 * rate, min(s1 * rate, n_frames)))
    return out


def slab_keypoints(q_off: np.ndarray, r: SlabRange):
    """(row range [a, b) of the CSR keypoint arrays, the slab's own offsets) of slab r."""
    a, b = int(q_off[r.s0]), int(q_off[r.s1])
    return a, b, (np.asarray(q_off[r.s0:r.s1 + 1], np.int64) - a).astype(np.int32)


def _hip_match(inp: _pl.SlabInputs, cfg: _pl.AlignConfig):
    m = _pl.match_stage(inp, cfg)
    return m.keep_bits, m.kp_ordered, m.counts  # counts: the per-frame log lines (VA:215-221)


def _hip_stages():
    """distributed.HIP_STAGES, with the match also handing back the per-frame counts."""
    import dataclasses

    from . import distributed as kdist

    return dataclasses.replace(kdist.HIP_STAGES, match=_hip_match)


def _on(t: torch.Tensor):
    """The device context of a slab's tensors (launches, allocations and the library's
    per-device context follow it); a no-op for CPU stand-ins."""
    return torch.cuda.device(t.device) if t.device.type == "cuda" else contextlib.nullcontext()


@dataclass
class SplitResult:
    aligned: List[torch.Tensor]   # per slab, on the slab's device: [f1 - f0, H, W(, C)] u16
    ranges: List[SlabRange]
    affines: np.ndarray           # [S * rate, 2, 3] (or [.., 3, 3]) after interpolation
    euclidean: np.ndarray
    skipped: List[int]
    interpolated: List[int]


def align_split(slabs: Sequence[_pl.SlabInputs], ranges: Sequence[SlabRange], cfg: _pl.AlignConfig,
                logger: Optional[logging.Logger] = None, impl=None) -> SplitResult:
    """The hot path over slabs that together hold every frame of one stack (``ranges``
    from split_frames, ``slabs[k]`` on any device: its full-rate frames, the template and
    its sample frames' keypoints).  Returns the per-slab aligned frames and the global
    affines / Euclidean transforms / skipped / interpolated lists of align_slab."""
    if len(slabs) != len(ranges) or not slabs:
        raise ValueError("align_split: one SlabRange per slab, at least one slab")
    impl = impl or _hip_stages()
    n_tpl = slabs[0].des_tpl.shape[0]
    n_sample = ranges[-1].s1
    # 1. match + vote of every slab, queued on every device before the host waits
    matched, counts = [], []
    for inp, r in zip(slabs, ranges):
        if inp.q_off.numel() - 1 != r.s1 - r.s0:
            raise ValueError("align_split: a slab's keypoint offsets do not match its SlabRange")
        with _on(inp.kp_tpl):
            keep_bits, kp_ordered, *cnt = impl.match(inp, cfg)
            matched.append((keep_bits, kp_ordered, impl.vote(keep_bits, n_tpl, r.s0)))
            counts.append(cnt[0] if cnt else None)
    if logger is not None and logger.isEnabledFor(logging.DEBUG):
        for c, r in zip(counts, ranges):
            if c is not None:
                _pl.log_frame_counts(logger, c.cpu().numpy(), r.s0)
    # 2. one merge of every slab's votes on the host
    votes = np.stack([v.cpu().numpy() for _, _, v in matched])
    choice = _pl.choose_consensus(votes, n_tpl, n_sample, cfg, logger)
    for inp, r in zip(slabs, ranges):
        if inp.frames.shape[0] != r.f1 - r.f0:
            raise ValueError("align_split: a slab's frames do not match its SlabRange")
    # 3. lookup + RANSAC of every slab.  Without temporal downsampling a frame with a model
    # keeps its own parameters through the post-processing (VA:143-145), so each slab's warp
    # is queued right behind its RANSAC with the parameters where RANSAC left them, and the
    # host post-processes while it runs; only the frames without a model (warped to zeros)
    # wait for the host's gap-filled maps.
    device_maps = impl.warp_params is not None and int(cfg.frame_downsample_rate) == 1
    fitted, aligned = [], []
    for inp, (keep_bits, kp_ordered, _) in zip(slabs, matched):
        with _on(inp.kp_tpl):
            cons = impl.lookup(keep_bits, n_tpl, choice)
            params = _to_host_async(impl.ransac(kp_ordered, inp.kp_tpl, cons, cfg))
            fitted.append((cons, params))
            if device_maps:
                aligned.append(impl.warp_params(inp.frames, params[0]))
    if logger is not None and logger.isEnabledFor(logging.INFO):
        for (cons, _), r in zip(fitted, ranges):
            _pl._log_low_counts(logger, np.diff(cons.pt_off), cfg, r.s0)
    # 4. the global post-processing, once
    params = np.concatenate([_host_array(p) for _, p in fitted])
    affines, skipped, interpolated, eu = _pl.postprocess_affines(params, cfg)
    # 5. the warp of every slab with its rows of the global maps (device maps: only the
    # frames without a model)
    if device_maps:
        redo = np.zeros(len(affines), bool)
        redo[np.asarray(skipped, dtype=np.int64)] = True
        for inp, r, out in zip(slabs, ranges, aligned):
            with _on(inp.kp_tpl):
                for a, b in _pl._runs(redo[r.f0:r.f1]):
                    out[a:b] = impl.warp(inp.frames[a:b], np.ascontiguousarray(affines[r.f0 + a:r.f0 + b]))
    else:
        for inp, r in zip(slabs, ranges):
            with _on(inp.kp_tpl):
                aligned.append(impl.warp(inp.frames, np.ascontiguousarray(affines[r.f0:r.f1])))
    return SplitResult(aligned, list(ranges), affines, eu, skipped, interpolated)


def _to_host_async(t: torch.Tensor):
    """(t, its host copy, an event after the copy): a device tensor is copied into pinned
    memory on the current stream without blocking the host; a host tensor is its own copy."""
    if t.device.type != "cuda":
        return t, t, None
    host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    host.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return t, host, ev


def _host_array(p) -> np.ndarray:
    _, host, ev = p
    if ev is not None:
        ev.synchronize()
    return host.numpy()


def visible_devices() -> List[int]:
    return list(range(torch.cuda.device_count()))


def split_to_devices(frames, ranges: Sequence[SlabRange], devices: Sequence[int]) -> List[torch.Tensor]:
    """Each slab's full-rate frames on its device: ``frames`` a host array [F, ...] (rows
    uploaded) or a device tensor (rows copied to the slab's device; no copy when it is
    already there)."""
    def upload(d, r):
        dev = torch.device("cuda", d)
        if isinstance(frames, torch.Tensor):
            return frames[r.f0:r.f1].to(dev).contiguous()
        with torch.cuda.device(dev):
            return torch.from_numpy(np.ascontiguousarray(frames[r.f0:r.f1])).to(dev)

    if isinstance(frames, torch.Tensor) or len(set(devices)) < 2:
        return [upload(d, r) for d, r in zip(devices, ranges)]
    # host frames to several devices: one uploading thread per slab, so the devices' PCIe links
    # run at once (a pageable copy blocks its caller; torch releases the GIL while it runs)
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=len(ranges)) as ex:
        return list(ex.map(upload, devices, ranges))


def make_slabs(parts: Sequence[torch.Tensor], ranges: Sequence[SlabRange], des_tpl: np.ndarray, kp_tpl: np.ndarray,
               kp_q: np.ndarray, des_q: np.ndarray, q_off: np.ndarray) -> List[_pl.SlabInputs]:
    """Slab inputs from each slab's frames (on its device, split_to_devices), the template
    (copied to every device) and the per-sample-frame CSR keypoints of the whole stack
    (kp_q [P, 2] f64, des_q [P, D], q_off [S + 1]), cut per slab."""
    if len(q_off) - 1 != (ranges[-1].s1 if ranges else 0):
        raise ValueError("keypoints must be given for every sample frame images[::rate]")
    slabs = []
    for fr, r in zip(parts, ranges):
        dev = fr.device
        a, b, off = slab_keypoints(q_off, r)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        slabs.append(_pl.SlabInputs(fr, t(des_tpl), t(np.asarray(kp_tpl, np.float64).reshape(-1, 2)),
                                    t(des_q[a:b]), t(np.asarray(kp_q[a:b], np.float64).reshape(-1, 2)), t(off), off))
    return slabs


def gather_aligned(res: SplitResult, out_device: Optional[torch.device] = None):
    """The aligned stack in one piece: on ``out_device`` (a device tensor), or on the host
    (numpy; each slab's frames copied into its slice of one pinned buffer)."""
    if out_device is not None:
        return torch.cat([a.to(out_device) for a in res.aligned])
    shape = (sum(a.shape[0] for a in res.aligned),) + tuple(res.aligned[0].shape[1:])
    host = torch.empty(shape, dtype=res.aligned[0].dtype, pin_memory=torch.cuda.is_available())
    for a, r in zip(res.aligned, res.ranges):
        host[r.f0:r.f1].copy_(a, non_blocking=True)
    if torch.cuda.is_available():
        for a in res.aligned:
            if a.device.type == "cuda":
                torch.cuda.current_stream(a.device).synchronize()
    return host.numpy()
