"""Batched hot-path stages on device-resident buffers (torch ROCm tensors as memory).

Each function launches HIP kernels from libkcmc.so through the C ABI
(include/kcmc.h) on the tensors' device and torch's current stream for that
device; nothing here computes on the CPU except the consensus, which is host
logic in the reference too (VA:224-286) and runs in native code.

Reference seams replaced (reference: /root/reference/VideoAligner.py):
  match_frames   <- _parallelize_i(_get_frame_keypoints, ...) matching part, VA:117-123 / VA:194-214
  consensus      <- _get_consensus_kps + _lookup_consensus_kps, VA:131-132 / VA:224-286
  ransac_rigid   <- _parallelize(_compute_euclidean_affine, ...), VA:137-142 / VA:288-323
  warp_affine    <- _parallelize(_apply_affine, images, affines), VA:150 / VA:455-458
"""
from __future__ import annotations

import contextlib
import ctypes
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib

_P = ctypes.c_void_p


def _ptr(t: Optional[torch.Tensor]):
    return _P(t.data_ptr()) if t is not None and t.numel() > 0 else _P(0)


def _np_ptr(a: Optional[np.ndarray]):
    return a.ctypes.data_as(_P) if a is not None and a.size > 0 else _P(0)


def _require(t: torch.Tensor, name: str, dtype: torch.dtype, device: torch.device, ndim: Optional[int] = None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim} dims, got shape {tuple(t.shape)}")


def _device_of(t: torch.Tensor) -> torch.device:
    if t.device.type != "cuda":
        raise _lib.KcmcLibraryError(
            "kcmc runs on the GPU only: pass device tensors (torch ROCm 'cuda' device); "
            "there is no CPU fallback for the alignment hot path"
        )
    return t.device


def _stream(device: torch.device, stream: Optional[int] = None):
    """The HIP stream of a launch: ``stream`` (a raw hipStream_t handle, as pipelines pass
    it) or torch's current stream on ``device``."""
    if stream is not None:
        return _P(stream)
    return _P(torch.cuda.current_stream(device).cuda_stream)


def on_stream(device: torch.device, stream: Optional[int] = None):
    """A context in which torch's current stream is ``stream`` (a raw hipStream_t handle)
    on ``device``, so that allocations and host reads made inside it are ordered with the
    launches made on that stream; a no-op for None (torch's current stream already is)."""
    if stream is None:
        return contextlib.nullcontext()
    return torch.cuda.stream(torch.cuda.ExternalStream(stream, device=device))


def memcpy_async(dst: int, src: int, nbytes: int, stream: int) -> None:
    """hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, stream) on raw pointers (pinned host
    <-> device transfers of the pipelines, without torch's per-copy dispatch)."""
    if nbytes > 0:
        _lib.check(_lib.load().kcmc_memcpy_async(_P(dst), _P(src), ctypes.c_size_t(nbytes), _P(stream)))


def _ctx(device: torch.device) -> _lib.Context:
    return _lib.context(device.index if device.index is not None else torch.cuda.current_device())


# ----------------------------------------------------------------------- K1
@dataclass
class MatchResult:
    idx: torch.Tensor          # [F, n_tpl, 2] i32  frame-keypoint index of best / 2nd best
    dist: torch.Tensor         # [F, n_tpl, 2] f32  OpenCV NORM_L2 distance
    kp_ordered: torch.Tensor   # [F, n_tpl, 2] f64  kp_query reordered to the template (VA:197-200)
    keep_bits: torch.Tensor    # [F, ceil(n_tpl/32)] i32 (bit pattern of u32) survivors of VA:202-213
    counts: torch.Tensor       # [F, 4] i32  numbers of the per-frame debug log (VA:215-221)


def _check_offsets(q_off_host: np.ndarray, n_frames: int) -> None:
    if q_off_host.shape != (n_frames + 1,) or q_off_host[0] != 0 or np.any(np.diff(q_off_host) < 0):
        raise ValueError("q_off must be [F+1] non-decreasing CSR offsets starting at 0")


def knn2_l2u8(des_tpl: torch.Tensor, des_q: torch.Tensor, q_off: torch.Tensor, max_nq: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """cv2.BFMatcher().knnMatch(des_tpl, des_q[frame], k=2) for every frame at once.
    uint8 descriptors (the reference's AKAZE/BRISK): exact integer distances, bit-exact
    with OpenCV's.  float32 (SIFT-style extension): the distance is DEFINED by this build
    as sqrtf of the sequentially fp64-accumulated sum of squares (oracle
    kcmc_oracle_knn2_l2f32); OpenCV's batchDistL2_32f accumulates in float in a
    build-dependent SIMD order, so near-ties (distances equal to ~1 ulp) can rank
    differently than with cv2 -- parity with OpenCV is unpinned for float descriptors."""
    dev = _device_of(des_tpl)
    f32 = des_tpl.dtype == torch.float32
    _require(des_tpl, "des_tpl", torch.float32 if f32 else torch.uint8, dev, 2)
    _require(des_q, "des_q", torch.float32 if f32 else torch.uint8, dev, 2)
    _require(q_off, "q_off", torch.int32, dev, 1)
    n_tpl, D = des_tpl.shape
    F = q_off.numel() - 1
    idx = torch.empty((F, n_tpl, 2), dtype=torch.int32, device=dev)
    dist = torch.empty((F, n_tpl, 2), dtype=torch.float32, device=dev)
    L = _lib.load()
    fn = L.kcmc_knn2_l2f32 if f32 else L.kcmc_knn2_l2u8
    _lib.check(fn(_ctx(dev).handle, _ptr(des_tpl), n_tpl, D, _ptr(des_q), _ptr(q_off), F, int(max_nq),
                  _ptr(idx), _ptr(dist), _stream(dev)))
    return idx, dist


def knn2_hamming(des_tpl: torch.Tensor, des_q: torch.Tensor, q_off: torch.Tensor, max_nq: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """cv2.BFMatcher(cv2.NORM_HAMMING).knnMatch(des_tpl, des_q[frame], k=2) for every frame
    (binary uint8 descriptors; opt-in, the reference's matcher is NORM_L2, VA:194)."""
    dev = _device_of(des_tpl)
    _require(des_tpl, "des_tpl", torch.uint8, dev, 2)
    _require(des_q, "des_q", torch.uint8, dev, 2)
    _require(q_off, "q_off", torch.int32, dev, 1)
    n_tpl, D = des_tpl.shape
    F = q_off.numel() - 1
    idx = torch.empty((F, n_tpl, 2), dtype=torch.int32, device=dev)
    dist = torch.empty((F, n_tpl, 2), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().kcmc_knn2_hamming(_ctx(dev).handle, _ptr(des_tpl), n_tpl, D, _ptr(des_q), _ptr(q_off), F,
                                             int(max_nq), _ptr(idx), _ptr(dist), _stream(dev)))
    return idx, dist


def match_frames(
    des_tpl: torch.Tensor,
    kp_tpl: torch.Tensor,
    des_q: torch.Tensor,
    kp_q: torch.Tensor,
    q_off: torch.Tensor,
    q_off_host: np.ndarray,
    ratio: float = 0.75,
    d_lo: float = 0.5,
    d_hi: float = 2.0,
    norm: str = "l2",
    stream: Optional[int] = None,
) -> MatchResult:
    """VA:194-214 for every frame: knn k=2 + reorder + ratio + median filters.
    uint8 descriptors (the reference's) or float32 (SIFT-style extension; its distance is
    this build's fp64-accumulated L2, not OpenCV's float accumulation, so near-tie order
    against cv2 is unpinned -- see knn2_l2u8); ``norm`` "hamming" (uint8 only) is the
    opt-in NORM_HAMMING matcher for binary descriptors."""
    dev, f32, n_tpl, D, F, max_nq = _match_args(des_tpl, kp_tpl, des_q, kp_q, q_off, q_off_host, norm)
    res = _match_result(dev, F, n_tpl)
    L = _lib.load()
    fn = L.kcmc_match_frames_f32 if f32 else (L.kcmc_match_frames_hamming if norm == "hamming" else L.kcmc_match_frames)
    _lib.check(fn(
        _ctx(dev).handle, _ptr(des_tpl), _ptr(kp_tpl), n_tpl, D, _ptr(des_q), _ptr(kp_q), _ptr(q_off), F,
        max_nq, float(ratio), float(d_lo), float(d_hi), _ptr(res.idx), _ptr(res.dist),
        _ptr(res.kp_ordered), _ptr(res.keep_bits), _ptr(res.counts), _stream(dev, stream)))
    return res


def _match_args(des_tpl, kp_tpl, des_q, kp_q, q_off, q_off_host, norm):
    """match_frames' argument checks: (device, float32?, n_tpl, D, F, max_nq)."""
    if norm not in ("l2", "hamming"):
        raise ValueError(f"norm must be 'l2' or 'hamming' (got {norm!r})")
    dev = _device_of(des_tpl)
    f32 = des_tpl.dtype == torch.float32
    if norm == "hamming" and f32:
        raise TypeError("NORM_HAMMING needs binary (uint8) descriptors")
    _require(des_tpl, "des_tpl", torch.float32 if f32 else torch.uint8, dev, 2)
    _require(kp_tpl, "kp_tpl", torch.float64, dev, 2)
    _require(des_q, "des_q", torch.float32 if f32 else torch.uint8, dev, 2)
    _require(kp_q, "kp_q", torch.float64, dev, 2)
    _require(q_off, "q_off", torch.int32, dev, 1)
    n_tpl, D = des_tpl.shape
    F = q_off.numel() - 1
    q_off_host = np.asarray(q_off_host)
    _check_offsets(q_off_host, F)
    nq = np.diff(q_off_host)
    if F and n_tpl and nq.min() < 2:
        bad = int(np.argmin(nq))
        raise ValueError(f"frame {bad} has {int(nq[bad])} keypoints; knnMatch(k=2) needs >= 2 (VA:203)")
    if kp_tpl.shape != (n_tpl, 2) or kp_q.shape[0] != des_q.shape[0] or int(q_off_host[-1]) > des_q.shape[0]:
        raise ValueError("keypoint/descriptor shapes disagree")
    return dev, f32, n_tpl, D, F, int(nq.max()) if F else 0


def _match_result(dev: torch.device, F: int, n_tpl: int, knn: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    idx, dist = knn if knn is not None else (torch.empty((F, n_tpl, 2), dtype=torch.int32, device=dev),
                                              torch.empty((F, n_tpl, 2), dtype=torch.float32, device=dev))
    return MatchResult(idx=idx, dist=dist,
                       kp_ordered=torch.empty((F, n_tpl, 2), dtype=torch.float64, device=dev),
                       keep_bits=torch.empty((F, (n_tpl + 31) // 32), dtype=torch.int32, device=dev),
                       counts=torch.empty((F, 4), dtype=torch.int32, device=dev))


def knn_frames(des_tpl: torch.Tensor, kp_tpl: torch.Tensor, des_q: torch.Tensor, kp_q: torch.Tensor,
               q_off: torch.Tensor, q_off_host: np.ndarray, norm: str = "l2",
               stream: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """match_frames in two parts, the first: the knn k=2 of every frame (VA:194-195) on
    ``stream``, idx / dist [F, n_tpl, 2]; filter_matches finishes it (on another stream
    ordered after this one, if wanted).  Same checks and results as match_frames."""
    dev, f32, n_tpl, D, F, max_nq = _match_args(des_tpl, kp_tpl, des_q, kp_q, q_off, q_off_host, norm)
    with on_stream(dev, stream):  # the outputs belong to the stream that writes them
        idx = torch.empty((F, n_tpl, 2), dtype=torch.int32, device=dev)
        dist = torch.empty((F, n_tpl, 2), dtype=torch.float32, device=dev)
    L = _lib.load()
    fn = L.kcmc_knn2_l2f32 if f32 else (L.kcmc_knn2_hamming if norm == "hamming" else L.kcmc_knn2_l2u8)
    _lib.check(fn(_ctx(dev).handle, _ptr(des_tpl), n_tpl, D, _ptr(des_q), _ptr(q_off), F, max_nq, _ptr(idx), _ptr(dist),
                  _stream(dev, stream)))
    return idx, dist


def filter_matches(knn: Tuple[torch.Tensor, torch.Tensor], kp_tpl: torch.Tensor, kp_q: torch.Tensor,
                   q_off: torch.Tensor, ratio: float = 0.75, d_lo: float = 0.5, d_hi: float = 2.0,
                   stream: Optional[int] = None) -> MatchResult:
    """The second part: VA:196-214 on knn_frames' (idx, dist) (kcmc_match_filter), on
    ``stream`` (its outputs are allocated there)."""
    idx, dist = knn
    dev = _device_of(idx)
    _require(idx, "idx", torch.int32, dev, 3)
    _require(dist, "dist", torch.float32, dev, 3)
    _require(kp_tpl, "kp_tpl", torch.float64, dev, 2)
    _require(kp_q, "kp_q", torch.float64, dev, 2)
    _require(q_off, "q_off", torch.int32, dev, 1)
    F, n_tpl = idx.shape[0], idx.shape[1]
    if dist.shape != idx.shape or idx.shape[2] != 2 or q_off.numel() != F + 1 or kp_tpl.shape != (n_tpl, 2):
        raise ValueError("knn results / keypoints shapes disagree")
    with on_stream(dev, stream):
        res = _match_result(dev, F, n_tpl, knn)
        if stream is not None:  # the knn tensors are read on this stream too
            cur = torch.cuda.current_stream(dev)
            idx.record_stream(cur)
            dist.record_stream(cur)
    _lib.check(_lib.load().kcmc_match_filter(
        _ctx(dev).handle, _ptr(idx), _ptr(dist), _ptr(kp_tpl), _ptr(kp_q), _ptr(q_off), F, n_tpl, float(ratio),
        float(d_lo), float(d_hi), _ptr(res.kp_ordered), _ptr(res.keep_bits), _ptr(res.counts), _stream(dev, stream)))
    return res


# ------------------------------------------------------------------ consensus
class Consensus:
    """The consensus of VA:224-286: ``order`` [n] i32 template indices in Counter.most_common
    order, ``votes`` [n] their counts, and the per-frame RANSAC point lists (VA:274) as CSR
    ``pt_off`` [F+1] / ``pt_idx`` [P] (template indices in CPython set-iteration order).
    The lists live on the host, on the device (``pt_off_dev`` / ``pt_idx_dev``, from the
    device lookup), or both; the host copies are made on first access."""

    def __init__(self, order: np.ndarray, votes: np.ndarray, pt_off: Optional[np.ndarray] = None,
                 pt_idx: Optional[np.ndarray] = None, pt_off_dev: Optional[torch.Tensor] = None,
                 pt_idx_dev: Optional[torch.Tensor] = None):
        self.order = order
        self.votes = votes
        self._pt_off = pt_off
        self._pt_idx = pt_idx
        self.pt_off_dev = pt_off_dev
        self.pt_idx_dev = pt_idx_dev

    @property
    def pt_off(self) -> np.ndarray:
        if self._pt_off is None:
            self._pt_off = self.pt_off_dev.cpu().numpy()
        return self._pt_off

    @property
    def pt_idx(self) -> np.ndarray:
        if self._pt_idx is None:
            n = int(self.pt_off[-1])
            self._pt_idx = self.pt_idx_dev[:n].cpu().numpy()
        return self._pt_idx


def consensus(keep_bits: np.ndarray, n_tpl: int, n_kp_global: int, n_min: int,
              frames: Optional[Tuple[int, int]] = None) -> Consensus:
    """VA:224-286 in native code with CPython set/Counter ordering.  With ``frames`` =
    (f_begin, f_end) the consensus still comes from every frame's bitmask but only the
    point lists of frames [f_begin, f_end) are made (pt_off starts at 0): a rank's share
    of a frame-sharded job."""
    kb = np.ascontiguousarray(keep_bits).view(np.uint32)
    F = kb.shape[0]
    if kb.shape != (F, (n_tpl + 31) // 32):
        raise ValueError("keep_bits must be [F, ceil(n_tpl/32)]")
    f0, f1 = (0, F) if frames is None else (int(frames[0]), int(frames[1]))
    if not 0 <= f0 <= f1 <= F:
        raise ValueError(f"frame range {frames} outside [0, {F}]")
    n_kp_global = int(n_kp_global)
    cons = np.zeros(max(n_kp_global, 1), np.int32)
    votes = np.zeros(max(n_kp_global, 1), np.int32)
    n_c = ctypes.c_int(0)
    pt_off = np.zeros(f1 - f0 + 1, np.int32)
    pt_idx = np.zeros(max((f1 - f0) * max(n_kp_global, 0), 1), np.int32)
    L = _lib.load()
    _lib.check(L.kcmc_consensus_slice(_np_ptr(kb), F, int(n_tpl), n_kp_global, int(n_min), f0, f1, _np_ptr(cons),
                                      _np_ptr(votes), ctypes.byref(n_c), _np_ptr(pt_off), _np_ptr(pt_idx)))
    n = n_c.value
    return Consensus(cons[:n].copy(), votes[:n].copy(), pt_off, pt_idx[: pt_off[-1]].copy())


def consensus_vote(keep_bits: torch.Tensor, n_tpl: int, frame_base: int = 0, out: Optional[torch.Tensor] = None,
                   stream: Optional[int] = None) -> torch.Tensor:
    """The vote part of the consensus (VA:239) on the device: [2, n_tpl] i64, row 0 the
    Counter count of every template over these frames, row 1 its first-occurrence key
    (frame_base + frame) << 32 | slot in that frame's CPython set table (INT64_MAX: never).
    Ranks' votes merge by summing counts and taking the min key (consensus_merge)."""
    dev = _device_of(keep_bits)
    _require(keep_bits, "keep_bits", torch.int32, dev, 2)
    if keep_bits.shape[1] != (n_tpl + 31) // 32:
        raise ValueError("keep_bits must be [F, ceil(n_tpl/32)]")
    if out is None:
        out = torch.empty((2, n_tpl), dtype=torch.int64, device=dev)
    _lib.check(_lib.load().kcmc_consensus_vote(_ctx(dev).handle, _ptr(keep_bits), keep_bits.shape[0], int(n_tpl),
                                               int(frame_base), _ptr(out), _stream(dev, stream)))
    return out


def consensus_vote_host(keep_bits: np.ndarray, n_tpl: int, frame_base: int = 0) -> np.ndarray:
    """consensus_vote of host bitmasks (native host code, same definition)."""
    kb = np.ascontiguousarray(keep_bits).view(np.uint32)
    if kb.ndim != 2 or kb.shape[1] != (n_tpl + 31) // 32:
        raise ValueError("keep_bits must be [F, ceil(n_tpl/32)]")
    out = np.empty((2, n_tpl), np.int64)
    _lib.check(_lib.load().kcmc_consensus_vote_host(_np_ptr(kb), kb.shape[0], int(n_tpl), int(frame_base),
                                                    _np_ptr(out)))
    return out


@dataclass
class ConsensusChoice:
    order: np.ndarray    # [nc] i32 Counter.most_common(n_kp_global) order
    votes: np.ndarray    # [nc] i32 counts
    pack: np.ndarray     # [>= nc + words] i32: set(consensus) iteration order, then its bitmask

    @property
    def nc(self) -> int:
        return len(self.order)

    @property
    def cons_iter(self) -> np.ndarray:
        return self.pack[: self.nc]


def consensus_merge(votes: np.ndarray, n_tpl: int, n_kp_global: int, n_min: int,
                    pack_out: Optional[np.ndarray] = None) -> ConsensusChoice:
    """Merge the votes of one or more ranks ([world, 2, n_tpl] or [2, n_tpl] i64):
    Counter.most_common(n_kp_global) (VA:240) + set(consensus) order (VA:248).  Raises
    VideoAligner.AlignmentError when fewer than n_min templates were voted (VA:241-244)."""
    v = np.ascontiguousarray(votes, dtype=np.int64)
    world = v.size // (2 * n_tpl) if n_tpl else 1
    if n_tpl and v.size != world * 2 * n_tpl:
        raise ValueError("votes must be [world, 2, n_tpl]")
    n_kp_global = int(n_kp_global)
    words = (n_tpl + 31) // 32
    order = np.zeros(max(n_kp_global, 1), np.int32)
    counts = np.zeros(max(n_kp_global, 1), np.int32)
    if pack_out is None:
        pack_out = np.zeros(n_kp_global + words, np.int32)
    elif pack_out.dtype != np.int32 or pack_out.size < n_kp_global + words or not pack_out.flags.c_contiguous:
        raise ValueError("pack_out must be a contiguous int32 array of >= n_kp_global + ceil(n_tpl/32) entries")
    n_c = ctypes.c_int(0)
    _lib.check(_lib.load().kcmc_consensus_merge(_np_ptr(v), int(world), int(n_tpl), n_kp_global, int(n_min),
                                                _np_ptr(order), _np_ptr(counts), ctypes.byref(n_c), _np_ptr(pack_out)))
    n = n_c.value
    return ConsensusChoice(order[:n].copy(), counts[:n].copy(), pack_out)


def consensus_lookup(keep_bits: torch.Tensor, n_tpl: int, pack_dev: torch.Tensor, nc: int,
                     stream: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The lookup part of the consensus (VA:274) on the device: every frame's
    list(consensus & frame_set) as CSR (pt_off [F+1], pt_idx [F*nc]) for RANSAC.
    pack_dev = ConsensusChoice.pack on the device."""
    dev = _device_of(keep_bits)
    _require(keep_bits, "keep_bits", torch.int32, dev, 2)
    _require(pack_dev, "pack_dev", torch.int32, dev, 1)
    F = keep_bits.shape[0]
    if keep_bits.shape[1] != (n_tpl + 31) // 32 or pack_dev.numel() < nc + keep_bits.shape[1] or not 0 <= nc <= n_tpl:
        raise ValueError("consensus_lookup: inconsistent shapes")
    L = _lib.load()
    pt_off = torch.empty(F + 1, dtype=torch.int32, device=dev)
    pt_idx = torch.empty(max(F * nc, 1), dtype=torch.int32, device=dev)
    # the set tables that do not fit in LDS (0 bytes for nc < 308: table size <= 1024)
    sb = int(L.kcmc_consensus_lookup_scratch_bytes(F, nc))
    scratch = torch.empty(sb, dtype=torch.uint8, device=dev) if sb > 0 else None
    _lib.check(L.kcmc_consensus_lookup(_ctx(dev).handle, _ptr(keep_bits), F, int(n_tpl), _ptr(pack_dev), int(nc),
                                       _ptr(pt_off), _ptr(pt_idx), _ptr(scratch), _stream(dev, stream)))
    return pt_off, pt_idx


def consensus_lookup_host(keep_bits: np.ndarray, n_tpl: int, cons_iter: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """consensus_lookup of host bitmasks (native host code)."""
    kb = np.ascontiguousarray(keep_bits).view(np.uint32)
    ci = np.ascontiguousarray(cons_iter, dtype=np.int32)
    F, nc = kb.shape[0], ci.size
    pt_off = np.zeros(F + 1, np.int32)
    pt_idx = np.zeros(max(F * nc, 1), np.int32)
    _lib.check(_lib.load().kcmc_consensus_lookup_host(_np_ptr(kb), F, int(n_tpl), _np_ptr(ci), nc, _np_ptr(pt_off),
                                                      _np_ptr(pt_idx)))
    return pt_off, pt_idx[: pt_off[-1]].copy()


def params_boundary(params: torch.Tensor, out: Optional[torch.Tensor] = None,
                    stream: Optional[int] = None) -> torch.Tensor:
    """[2 + 2E] f64: the first and last frame of params [F, ...] without NaN (-1: none) and
    their parameters -- what the neighbouring ranks need for NaN-gap filling (VA:347-407)."""
    dev = _device_of(params)
    _require(params, "params", torch.float64, dev)
    F = params.shape[0]
    E = int(params[0].numel()) if F else int(np.prod(params.shape[1:]))
    if out is None:
        out = torch.empty(2 + 2 * E, dtype=torch.float64, device=dev)
    _lib.check(_lib.load().kcmc_params_boundary(_ctx(dev).handle, _ptr(params), F, E, _ptr(out), _stream(dev, stream)))
    return out


def hypothesis_table(n: int, trials: int = 1000, seed: int = 42, min_samples: int = 2) -> np.ndarray:
    """The per-trial samples skimage 0.18.3's ransac draws (legacy MT19937)."""
    out = np.empty((trials, min_samples), np.int32)
    _lib.check(_lib.load().kcmc_hypothesis_table(int(n), int(trials), int(seed) & 0xFFFFFFFF, int(min_samples),
                                                 _np_ptr(out)))
    return out


# ----------------------------------------------------------------------- K2
@dataclass
class RansacResult:
    params: torch.Tensor       # [F, 2, 3] f64 (NaN where the reference returns NaN)
    inliers: torch.Tensor      # [P] u8 inlier mask of the best hypothesis (CSR like the points)
    n_inliers: torch.Tensor    # [F] i32
    best_trial: torch.Tensor   # [F] i32 (-1: none)


def ransac_rigid(
    src: torch.Tensor,
    dst: torch.Tensor,
    pt_off: torch.Tensor,
    pt_off_host: np.ndarray,
    pt_idx: Optional[torch.Tensor] = None,
    src_frame_stride: int = 0,
    trials: int = 1000,
    residual_threshold: float = 2.0,
    spatial_rate: float = 1.0,
    n_skip: int = 3,
    seed: int = 42,
    min_samples: int = 2,
) -> RansacResult:
    """skimage ransac(EuclideanTransform) per frame (VA:288-323), all frames in one launch.

    With ``pt_idx``: point k of frame f is src[f*src_frame_stride + pt_idx[k]] /
    dst[pt_idx[k]] (src = kp_ordered [F*n_tpl, 2], dst = template keypoints).
    """
    dev = _device_of(src)
    _require(src, "src", torch.float64, dev, 2)
    _require(dst, "dst", torch.float64, dev, 2)
    _require(pt_off, "pt_off", torch.int32, dev, 1)
    if pt_idx is not None:
        _require(pt_idx, "pt_idx", torch.int32, dev, 1)
    if min_samples != 2:
        raise ValueError("rigid RANSAC uses min_samples=2 (EuclideanTransform, VA:312)")
    F = pt_off.numel() - 1
    pt_off_host = np.asarray(pt_off_host)
    _check_offsets(pt_off_host, F)
    ns = np.diff(pt_off_host)
    # skimage raises when a frame is not skipped but has N <= min_samples (fit.py:798-799)
    bad = (ns >= n_skip) & (ns <= min_samples)
    if bad.any():
        raise ValueError("`min_samples` must be in range (0, <number-of-samples>)")
    max_n = int(ns.max()) if F else 0
    P = int(pt_off_host[-1]) if F else 0
    res = RansacResult(
        params=torch.empty((F, 2, 3), dtype=torch.float64, device=dev),
        inliers=torch.empty((max(P, 0),), dtype=torch.uint8, device=dev),
        n_inliers=torch.empty((F,), dtype=torch.int32, device=dev),
        best_trial=torch.empty((F,), dtype=torch.int32, device=dev),
    )
    if F == 0:
        return res
    ctx = _ctx(dev)
    L = _lib.load()
    n_run = np.unique(ns[ns >= max(int(n_skip), 3)]).astype(np.int32)
    _lib.check(L.kcmc_ransac_prepare(ctx.handle, _np_ptr(n_run), int(n_run.size), int(trials),
                                     int(seed) & 0xFFFFFFFF))
    _lib.check(L.kcmc_ransac_rigid(
        ctx.handle, _ptr(src), _ptr(dst), _ptr(pt_idx), _ptr(pt_off), int(src_frame_stride), F, max_n, int(trials),
        float(residual_threshold), float(spatial_rate), int(n_skip), _ptr(res.params), _ptr(res.inliers),
        _ptr(res.n_inliers), _ptr(res.best_trial), _stream(dev)))
    return res


def ransac_model(
    src: torch.Tensor,
    dst: torch.Tensor,
    pt_off: torch.Tensor,
    pt_off_host: np.ndarray,
    model: str = "affine",
    pt_idx: Optional[torch.Tensor] = None,
    src_frame_stride: int = 0,
    trials: int = 1000,
    residual_threshold: float = 2.0,
    spatial_rate: float = 1.0,
    n_skip: int = 3,
    seed: int = 42,
) -> RansacResult:
    """skimage ransac with AffineTransform (min_samples 3) or ProjectiveTransform
    (min_samples 4) per frame, all frames in one launch (the extension behind BASELINE
    configs 3-5; same call shape as VA:309-316).  params: [F, 3, 3] f64.

    Frames with n_skip <= N <= min_samples raise ValueError like skimage
    (fit.py:798-799); frames with N < n_skip get NaN (VA:306-307)."""
    if model not in ("affine", "projective"):
        raise ValueError(f"model must be 'affine' or 'projective' (got {model!r}); rigid: ransac_rigid")
    dev = _device_of(src)
    _require(src, "src", torch.float64, dev, 2)
    _require(dst, "dst", torch.float64, dev, 2)
    _require(pt_off, "pt_off", torch.int32, dev, 1)
    if pt_idx is not None:
        _require(pt_idx, "pt_idx", torch.int32, dev, 1)
    ms = _lib.MODEL_MIN_SAMPLES[model]
    F = pt_off.numel() - 1
    pt_off_host = np.asarray(pt_off_host)
    _check_offsets(pt_off_host, F)
    ns = np.diff(pt_off_host)
    bad = (ns >= n_skip) & (ns <= ms)
    if bad.any():
        raise ValueError("`min_samples` must be in range (0, <number-of-samples>)")
    max_n = int(ns.max()) if F else 0
    P = int(pt_off_host[-1]) if F else 0
    res = RansacResult(
        params=torch.empty((F, 3, 3), dtype=torch.float64, device=dev),
        inliers=torch.empty((max(P, 0),), dtype=torch.uint8, device=dev),
        n_inliers=torch.empty((F,), dtype=torch.int32, device=dev),
        best_trial=torch.empty((F,), dtype=torch.int32, device=dev),
    )
    if F == 0:
        return res
    ctx = _ctx(dev)
    L = _lib.load()
    n_run = np.unique(ns[ns >= max(int(n_skip), ms + 1)]).astype(np.int32)
    _lib.check(L.kcmc_ransac_prepare_samples(ctx.handle, ms, _np_ptr(n_run), int(n_run.size), int(trials),
                                             int(seed) & 0xFFFFFFFF))
    _lib.check(L.kcmc_ransac_model(
        ctx.handle, _lib.MODEL_IDS[model], _ptr(src), _ptr(dst), _ptr(pt_idx), _ptr(pt_off), int(src_frame_stride), F,
        max_n, int(trials), float(residual_threshold), float(spatial_rate), int(n_skip), _ptr(res.params),
        _ptr(res.inliers), _ptr(res.n_inliers), _ptr(res.best_trial), _stream(dev)))
    return res


def ransac_prepare_range(device, model: str, n_lo: int, n_hi: int, trials: int = 1000, seed: int = 42) -> None:
    """Make the hypothesis tables of every point count in [n_lo, n_hi] current on the
    device (the device lookup's point counts are not seen by the host; every count a frame
    can have is ready).  Called before every device-list RANSAC: the context keeps ONE
    (trials, seed) table set per min_samples, and another caller on the same context
    (ransac_rigid / ransac_model, or an aligner with another RANDOM_SEED) may have
    replaced it since; the C side regenerates only the counts it lacks and re-uploads
    only when the set changed, so a repeat call is one host loop over the range."""
    dev = torch.device(device)
    ctx = _ctx(dev)
    ms = _lib.MODEL_MIN_SAMPLES[model]
    n_lo = max(int(n_lo), ms + 1, 3)
    if int(n_hi) < n_lo:
        return
    n_run = np.arange(n_lo, int(n_hi) + 1, dtype=np.int32)
    L = _lib.load()
    seed = int(seed) & 0xFFFFFFFF
    if ms == 2:
        _lib.check(L.kcmc_ransac_prepare(ctx.handle, _np_ptr(n_run), int(n_run.size), int(trials), seed))
    else:
        _lib.check(L.kcmc_ransac_prepare_samples(ctx.handle, ms, _np_ptr(n_run), int(n_run.size), int(trials), seed))


def ransac_lists(model: str, src: torch.Tensor, dst: torch.Tensor, pt_off: torch.Tensor, pt_idx: torch.Tensor,
                 src_frame_stride: int, max_n: int, trials: int = 1000, residual_threshold: float = 2.0,
                 spatial_rate: float = 1.0, n_skip: int = 3, stream: Optional[int] = None) -> RansacResult:
    """RANSAC of every frame on device point lists whose sizes the host does not know
    (the device consensus lookup): max_n bounds every frame's point count (n_kp_global) and
    the tables of every count in [n_skip, max_n] must be ready (ransac_prepare_range).
    params [F, 2, 3] (euclidean) or [F, 3, 3] (affine / projective), as ransac_rigid /
    ransac_model."""
    dev = _device_of(src)
    F = pt_off.numel() - 1
    P = pt_idx.numel()
    res = RansacResult(
        params=torch.empty((F, 2, 3) if model == "euclidean" else (F, 3, 3), dtype=torch.float64, device=dev),
        inliers=torch.empty((max(P, 1),), dtype=torch.uint8, device=dev),
        n_inliers=torch.empty((F,), dtype=torch.int32, device=dev),
        best_trial=torch.empty((F,), dtype=torch.int32, device=dev),
    )
    if F == 0:
        return res
    L = _lib.load()
    ctx = _ctx(dev).handle
    st = _stream(dev, stream)
    if model == "euclidean":
        _lib.check(L.kcmc_ransac_rigid(
            ctx, _ptr(src), _ptr(dst), _ptr(pt_idx), _ptr(pt_off), int(src_frame_stride), F, int(max_n), int(trials),
            float(residual_threshold), float(spatial_rate), int(n_skip), _ptr(res.params), _ptr(res.inliers),
            _ptr(res.n_inliers), _ptr(res.best_trial), st))
    else:
        _lib.check(L.kcmc_ransac_model(
            ctx, _lib.MODEL_IDS[model], _ptr(src), _ptr(dst), _ptr(pt_idx), _ptr(pt_off), int(src_frame_stride), F,
            int(max_n), int(trials), float(residual_threshold), float(spatial_rate), int(n_skip), _ptr(res.params),
            _ptr(res.inliers), _ptr(res.n_inliers), _ptr(res.best_trial), st))
    return res


# ----------------------------------------------------------------------- K3
def warp_affine_u16(frames: torch.Tensor, affines: torch.Tensor, out: Optional[torch.Tensor] = None,
                    inverse_map: bool = False, stream: Optional[int] = None) -> torch.Tensor:
    """cv2.warpAffine(frame, M, (W, H), INTER_LINEAR) for every frame (VA:458).

    frames [F, H, W] or [F, H, W, C] uint16 on the device; affines [F, 2, 3] f64.
    """
    dev = _device_of(frames)
    if frames.dtype != torch.uint16:
        raise TypeError(f"frames: expected torch.uint16, got {frames.dtype}")
    if frames.dim() not in (3, 4):
        raise ValueError("frames must be [F, H, W] or [F, H, W, C]")
    _require(frames, "frames", torch.uint16, dev)
    _require(affines, "affines", torch.float64, dev, 3)
    F, H, W = frames.shape[:3]
    C = 1 if frames.dim() == 3 else frames.shape[3]
    if affines.shape != (F, 2, 3):
        raise ValueError(f"affines must be [{F}, 2, 3], got {tuple(affines.shape)}")
    if out is None:
        out = torch.empty_like(frames)
    else:
        _require(out, "out", torch.uint16, dev)
        if out.shape != frames.shape:
            raise ValueError("out must have the shape of frames")
    L = _lib.load()
    _lib.check(L.kcmc_warp_affine_u16(_ctx(dev).handle, _ptr(frames), _ptr(out), _ptr(affines), F, H, W, C,
                                      int(bool(inverse_map)), _stream(dev, stream)))
    return out


def warp_perspective_u16(frames: torch.Tensor, homographies: torch.Tensor, out: Optional[torch.Tensor] = None,
                         inverse_map: bool = False, stream: Optional[int] = None) -> torch.Tensor:
    """cv2.warpPerspective(frame, H, (W, H), INTER_LINEAR) for every frame (the warp of
    the homography extension).  frames [F, H, W] or [F, H, W, C] uint16; homographies
    [F, 3, 3] f64 (forward maps, frame -> template, as RANSAC returns them)."""
    dev = _device_of(frames)
    if frames.dtype != torch.uint16:
        raise TypeError(f"frames: expected torch.uint16, got {frames.dtype}")
    if frames.dim() not in (3, 4):
        raise ValueError("frames must be [F, H, W] or [F, H, W, C]")
    _require(frames, "frames", torch.uint16, dev)
    _require(homographies, "homographies", torch.float64, dev, 3)
    F, H, W = frames.shape[:3]
    C = 1 if frames.dim() == 3 else frames.shape[3]
    if homographies.shape != (F, 3, 3):
        raise ValueError(f"homographies must be [{F}, 3, 3], got {tuple(homographies.shape)}")
    if out is None:
        out = torch.empty_like(frames)
    else:
        _require(out, "out", torch.uint16, dev)
        if out.shape != frames.shape:
            raise ValueError("out must have the shape of frames")
    L = _lib.load()
    _lib.check(L.kcmc_warp_perspective_u16(_ctx(dev).handle, _ptr(frames), _ptr(out), _ptr(homographies), F, H, W, C,
                                           int(bool(inverse_map)), _stream(dev, stream)))
    return out


def _warp_shape(frames_shape) -> Tuple[int, int, int, int]:
    if len(frames_shape) not in (3, 4):
        raise ValueError("frames must be [F, H, W] or [F, H, W, C]")
    F, H, W = (int(v) for v in frames_shape[:3])
    return F, H, W, 1 if len(frames_shape) == 3 else int(frames_shape[3])


# ------------------------------------------------------------ f2: normalisation
def _numpy_linear_percentile(n: int, q: float, value_at) -> np.float64:
    """np.percentile(a, q) (default 'linear' method) of a flattened integer array of n
    elements, given value_at(rank) = the rank-th smallest element: numpy's virtual
    index (n - 1) * q' with q' = q/100 (numpy >= 1.22 'linear'), floor/next ranks
    clipped to the array, and its _lerp (a + (b-a)*t, or b - (b-a)*(1-t) when t >= 0.5),
    evaluated with the same float64 operations."""
    qq = np.true_divide(np.float64(q), 100)
    vi = (n - 1) * qq
    prev = np.floor(vi)
    if vi >= n - 1:
        lo = hi = n - 1
    elif vi < 0:
        lo = hi = 0
    else:
        lo, hi = int(prev), int(prev) + 1
    gamma = np.float64(vi - prev)
    a, b = np.uint16(value_at(lo)), np.uint16(value_at(hi))
    diff = np.subtract(b, a)
    if gamma >= 0.5:
        return np.float64(np.subtract(b, diff * (1 - gamma)))
    return np.float64(np.add(a, diff * gamma))


def _aligned16(t: torch.Tensor) -> torch.Tensor:
    """``t`` itself when its data is 16-byte aligned (the histogram / LUT kernels read 16
    bytes per lane), else an aligned copy: a frame slab that starts mid-allocation (a view
    of a stack whose frame size is not a multiple of 16 bytes)."""
    return t if t.data_ptr() % 16 == 0 else t.clone()


def brightest_px(frames, percentile: float = 99.99) -> np.float64:
    """VA:479-482 on the device: np.percentile(images, 99.99) of a uint16 stack, exact
    (two order statistics from two histogram passes, numpy's interpolation on the host).
    ``frames``: one device tensor, or the slabs of one stack on several devices (their
    histograms are summed: the percentile of the whole stack)."""
    parts = [frames] if isinstance(frames, torch.Tensor) else list(frames)
    for p in parts:
        _require(p, "frames", torch.uint16, _device_of(p))
    parts = [_aligned16(p) for p in parts]
    n = sum(p.numel() for p in parts)
    if n == 0:
        raise ValueError("percentile of an empty stack")
    L = _lib.load()

    def histogram(shift: int, hb: int) -> np.ndarray:
        hs = []
        for p in parts:  # queued on every device before the first host read
            dev = _device_of(p)
            with torch.cuda.device(dev):  # the launch, its workspace and h on the part's device
                h = torch.empty(256, dtype=torch.int64, device=dev)
                if p.numel():
                    _lib.check(L.kcmc_histogram_u16(_ctx(dev).handle, _ptr(p), p.numel(), shift, hb, _ptr(h),
                                                    _stream(dev)))
                else:
                    h.zero_()
            hs.append(h)
        return np.sum([h.cpu().numpy() for h in hs], axis=0)

    coarse = np.cumsum(histogram(8, -1))
    fine_cache = {}

    def value_at(rank: int) -> int:
        hb = int(np.searchsorted(coarse, rank, side="right"))
        if hb not in fine_cache:
            fine_cache[hb] = np.cumsum(histogram(0, hb))
        below = int(coarse[hb - 1]) if hb > 0 else 0
        lb = int(np.searchsorted(fine_cache[hb], rank - below, side="right"))
        return (hb << 8) | lb

    return _numpy_linear_percentile(n, percentile, value_at)


def max_scale_lut(brightest: float, max_px: int = 255, dtype=np.uint8) -> np.ndarray:
    """The reference's max-scaling (VA:490) evaluated once for every uint16 value."""
    v = np.arange(65536, dtype=np.uint16)
    return np.clip(v / brightest * max_px, a_min=0, a_max=max_px).astype(dtype)


def max_scale_u8(frames: torch.Tensor, brightest: float, out: Optional[torch.Tensor] = None,
                 max_px: int = 255) -> torch.Tensor:
    """VA:484-492 on the device: np.clip(frames / brightest * 255, 0, 255).astype(uint8)."""
    dev = _device_of(frames)
    _require(frames, "frames", torch.uint16, dev)
    if out is None:
        out = torch.empty(frames.shape, dtype=torch.uint8, device=dev)
    else:
        _require(out, "out", torch.uint8, dev)
        if out.shape != frames.shape:
            raise ValueError("out must have the shape of frames")
    lut = torch.from_numpy(max_scale_lut(float(brightest), max_px)).to(dev)
    res = out if out.data_ptr() % 16 == 0 else torch.empty_like(out)
    _lib.check(_lib.load().kcmc_lut_u16_to_u8(_ctx(dev).handle, _ptr(_aligned16(frames)), frames.numel(), _ptr(lut),
                                              _ptr(res), _stream(dev)))
    if res is not out:
        out.copy_(res)
    return out


# ------------------------------------------------------------ f4: pyrDown
def pyr_down_u8(frames_u8: torch.Tensor, dstsize=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cv2.pyrDown(frame, dstsize=dstsize) of every frame of a uint8 stack [F, H, W]
    (VA:501-503) on the device.  dstsize is (width, height) like OpenCV; None or an
    empty size gives ((W + 1) // 2, (H + 1) // 2).  ValueError where OpenCV's size
    assertion (|2 w - W| <= 2, |2 h - H| <= 2) fails."""
    dev = _device_of(frames_u8)
    _require(frames_u8, "frames_u8", torch.uint8, dev)
    if frames_u8.dim() != 3:
        raise ValueError("frames_u8 must be [F, H, W]")
    F, H, W = frames_u8.shape
    if H == 0 or W == 0:
        raise ValueError("pyrDown: ssize.width > 0 && ssize.height > 0")
    dw, dh = ((W + 1) // 2, (H + 1) // 2) if dstsize is None or min(dstsize) <= 0 else (int(dstsize[0]), int(dstsize[1]))
    if abs(2 * dw - W) > 2 or abs(2 * dh - H) > 2:
        raise ValueError("pyrDown: std::abs(dsize.width*2 - ssize.width) <= 2 && "
                         "std::abs(dsize.height*2 - ssize.height) <= 2")
    if out is None:
        out = torch.empty((F, dh, dw), dtype=torch.uint8, device=dev)
    else:
        _require(out, "out", torch.uint8, dev)
        if tuple(out.shape) != (F, dh, dw):
            raise ValueError("out must be [F, dst_h, dst_w]")
    _lib.check(_lib.load().kcmc_pyr_down_u8(_ctx(dev).handle, _ptr(frames_u8), F, H, W, _ptr(out), dh, dw,
                                            _stream(dev)))
    return out


# ------------------------------------------------------------ f1: detection
@dataclass
class Keypoints:
    kp: torch.Tensor      # [F, n_features, 2] f64 (x, y); rows >= count[f] undefined
    des: torch.Tensor     # [F, n_features, 32] u8
    count: torch.Tensor   # [F] i32


def detect_orb(frames_u8: torch.Tensor, params=None) -> Keypoints:
    """The build's ORB-style detector (csrc/orb.hip) for every frame of a uint8 stack:
    replaces detector.detectAndCompute (VA:114-116, VA:190-192) on the device."""
    from . import orb

    params = params or orb.OrbParams()
    dev = _device_of(frames_u8)
    _require(frames_u8, "frames_u8", torch.uint8, dev)
    if frames_u8.dim() == 2:
        frames_u8 = frames_u8.unsqueeze(0)
    if frames_u8.dim() != 3:
        raise ValueError("frames_u8 must be [F, H, W] or [H, W]")
    F, H, W = frames_u8.shape
    N = int(params.n_features)
    res = Keypoints(kp=torch.empty((F, N, 2), dtype=torch.float64, device=dev),
                    des=torch.empty((F, N, 32), dtype=torch.uint8, device=dev),
                    count=torch.empty((F,), dtype=torch.int32, device=dev))
    pattern = torch.from_numpy(orb.rotated_patterns()).to(dev)
    cs = torch.from_numpy(orb.bin_edges()).to(dev)
    _lib.check(_lib.load().kcmc_orb_detect(
        _ctx(dev).handle, _ptr(frames_u8), F, H, W, int(params.fast_threshold), N, float(params.harris_k),
        int(params.edge), _ptr(pattern), _ptr(cs), _ptr(res.kp), _ptr(res.des), _ptr(res.count), _stream(dev)))
    return res


def keypoints_csr(k: Keypoints):
    """Per-frame keypoints -> the matcher's CSR layout: (kp [P, 2] f64, des [P, 32] u8,
    q_off (device i32 [F+1]), q_off_host)."""
    counts = k.count.cpu().numpy().astype(np.int64)
    F, N = k.kp.shape[:2]
    q_off = np.zeros(F + 1, np.int32)
    q_off[1:] = np.cumsum(counts)
    if F and (counts == N).all():  # every frame full (the common case): the arrays as they are
        kp = k.kp.reshape(F * N, 2).contiguous()
        des = k.des.reshape(F * N, 32).contiguous()
    else:  # the first count[f] rows of every frame, in frame order (compacted on the device)
        live = torch.arange(N, device=k.kp.device)[None, :] < k.count.to(torch.int64)[:, None]
        kp = k.kp[live].contiguous()
        des = k.des[live].contiguous()
    return kp, des, torch.from_numpy(q_off).to(k.kp.device), q_off
