"""ctypes binding of libkcmc.so (the C ABI declared in include/kcmc.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be
loaded, every entry point raises ``KcmcLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

from . import build as _build

KCMC_OK = 0
KCMC_EINVAL = 1
KCMC_EHIP = 2
KCMC_ENOMEM = 3
KCMC_EUNSUPPORTED = 4
KCMC_EALIGN = 5
ABI_VERSION = 2

# Every symbol include/kcmc.h declares (checked by tests/test_capi.py).
EXPORTED_SYMBOLS = (
    "kcmc_abi_version",
    "kcmc_last_error",
    "kcmc_memcpy_async",
    "kcmc_create",
    "kcmc_destroy",
    "kcmc_knn2_l2u8",
    "kcmc_match_frames",
    "kcmc_match_filter",
    "kcmc_knn2_l2f32",
    "kcmc_match_frames_f32",
    "kcmc_knn2_hamming",
    "kcmc_match_frames_hamming",
    "kcmc_consensus",
    "kcmc_consensus_slice",
    "kcmc_consensus_vote",
    "kcmc_consensus_vote_host",
    "kcmc_consensus_merge",
    "kcmc_consensus_lookup_scratch_bytes",
    "kcmc_consensus_lookup",
    "kcmc_consensus_lookup_host",
    "kcmc_params_boundary",
    "kcmc_hypothesis_table",
    "kcmc_ransac_prepare",
    "kcmc_ransac_rigid",
    "kcmc_ransac_prepare_samples",
    "kcmc_ransac_model",
    "kcmc_warp_affine_u16",
    "kcmc_warp_perspective_u16",
    "kcmc_histogram_u16",
    "kcmc_lut_u16_to_u8",
    "kcmc_orb_detect",
    "kcmc_pyr_down_u8",
)

KCMC_MODEL_EUCLIDEAN = 0
KCMC_MODEL_AFFINE = 1
KCMC_MODEL_PROJECTIVE = 2
MODEL_IDS = {"euclidean": KCMC_MODEL_EUCLIDEAN, "affine": KCMC_MODEL_AFFINE, "projective": KCMC_MODEL_PROJECTIVE}
MODEL_MIN_SAMPLES = {"euclidean": 2, "affine": 3, "projective": 4}


class KcmcLibraryError(RuntimeError):
    """libkcmc.so is missing or failed to load (no CPU fallback exists)."""


class KcmcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"kcmc error {code}: {msg}")
        self.code = code
        self.msg = msg


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None

P = ctypes.c_void_p
I = ctypes.c_int
D = ctypes.c_double
U32 = ctypes.c_uint32
LL = ctypes.c_longlong

_SIGNATURES = {
    "kcmc_abi_version": ([], I),
    "kcmc_last_error": ([], ctypes.c_char_p),
    "kcmc_memcpy_async": ([P, P, ctypes.c_size_t, P], I),
    "kcmc_create": ([I, ctypes.POINTER(P)], I),
    "kcmc_destroy": ([P], I),
    "kcmc_knn2_l2u8": ([P, P, I, I, P, P, I, I, P, P, P], I),
    "kcmc_match_frames": ([P, P, P, I, I, P, P, P, I, I, D, D, D, P, P, P, P, P, P], I),
    "kcmc_match_filter": ([P, P, P, P, P, P, I, I, D, D, D, P, P, P, P], I),
    "kcmc_knn2_l2f32": ([P, P, I, I, P, P, I, I, P, P, P], I),
    "kcmc_match_frames_f32": ([P, P, P, I, I, P, P, P, I, I, D, D, D, P, P, P, P, P, P], I),
    "kcmc_knn2_hamming": ([P, P, I, I, P, P, I, I, P, P, P], I),
    "kcmc_match_frames_hamming": ([P, P, P, I, I, P, P, P, I, I, D, D, D, P, P, P, P, P, P], I),
    "kcmc_consensus": ([P, I, I, I, I, P, P, P, P, P], I),
    "kcmc_consensus_slice": ([P, I, I, I, I, I, I, P, P, P, P, P], I),
    "kcmc_consensus_vote": ([P, P, I, I, LL, P, P], I),
    "kcmc_consensus_vote_host": ([P, I, I, LL, P], I),
    "kcmc_consensus_merge": ([P, I, I, I, I, P, P, P, P], I),
    "kcmc_consensus_lookup_scratch_bytes": ([I, I], LL),
    "kcmc_consensus_lookup": ([P, P, I, I, P, I, P, P, P, P], I),
    "kcmc_consensus_lookup_host": ([P, I, I, P, I, P, P], I),
    "kcmc_params_boundary": ([P, P, I, I, P, P], I),
    "kcmc_hypothesis_table": ([I, I, U32, I, P], I),
    "kcmc_ransac_prepare": ([P, P, I, I, U32], I),
    "kcmc_ransac_rigid": ([P, P, P, P, P, I, I, I, I, D, D, I, P, P, P, P, P], I),
    "kcmc_ransac_prepare_samples": ([P, I, P, I, I, U32], I),
    "kcmc_ransac_model": ([P, I, P, P, P, P, I, I, I, I, D, D, I, P, P, P, P, P], I),
    "kcmc_warp_affine_u16": ([P, P, P, P, I, I, I, I, I, P], I),
    "kcmc_warp_perspective_u16": ([P, P, P, P, I, I, I, I, I, P], I),
    "kcmc_histogram_u16": ([P, P, ctypes.c_ulonglong, I, I, P, P], I),
    "kcmc_lut_u16_to_u8": ([P, P, ctypes.c_ulonglong, P, P, P], I),
    "kcmc_orb_detect": ([P, P, I, I, I, I, I, D, I, P, P, P, P, P, P], I),
    "kcmc_pyr_down_u8": ([P, P, I, I, I, P, I, I, P], I),
}


def _alt_lib() -> str:
    """KCMC_LIB_PATH: another build of the same library (same-box A/B runs of tools/ and the
    debug sentinel build), honoured only together with the explicit test-only switch
    KCMC_TEST_ONLY_ALT_LIB=1; set alone it is an error, not a silent swap of the product."""
    alt = os.environ.get("KCMC_LIB_PATH")
    if not alt:
        return ""
    if os.environ.get("KCMC_TEST_ONLY_ALT_LIB") != "1":
        raise KcmcLibraryError("KCMC_LIB_PATH is a test-only override: set KCMC_TEST_ONLY_ALT_LIB=1 as well to "
                               "load an alternative build")
    return alt


def lib_path() -> str:
    return _alt_lib() or _build.LIB_PATH


def load(auto_build: bool = True) -> ctypes.CDLL:
    """Load libkcmc.so (building it with hipcc first when allowed and stale)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        alt = _alt_lib()
        path = alt or _build.LIB_PATH
        if alt:
            import warnings

            warnings.warn(f"KCMC_LIB_PATH set: loading {path} (an A/B build; no auto-build, entry points it lacks "
                          "stay unbound and fail when called)", RuntimeWarning, stacklevel=2)
        if auto_build and os.environ.get("KCMC_NO_BUILD", "0") != "1" and not alt:
            try:
                if not _build.up_to_date():
                    _build.build()
            except Exception as e:  # pragma: no cover - only when hipcc is broken
                if not os.path.exists(path):
                    raise KcmcLibraryError(f"cannot build {path}: {e}") from e
        if not os.path.exists(path):
            raise KcmcLibraryError(
                f"{path} not found: build it with `python -m kcmc_amd.build` (hipcc, gfx950). "
                "There is no CPU fallback for the alignment hot path."
            )
        try:
            L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise KcmcLibraryError(f"failed to load {path}: {e}") from e
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                if alt:  # an older A/B build: its missing entries stay unbound
                    continue
                raise KcmcLibraryError(f"{path}: missing symbol {name} (stale build?)")
            fn.argtypes = args
            fn.restype = res
        if L.kcmc_abi_version() != ABI_VERSION:
            raise KcmcLibraryError(f"{path}: ABI version {L.kcmc_abi_version()} != {ABI_VERSION}")
        _lib = L
        return L


def check(rc: int) -> None:
    if rc != KCMC_OK:
        msg = load().kcmc_last_error().decode(errors="replace")
        if rc == KCMC_EINVAL:
            raise ValueError(msg)
        if rc == KCMC_EALIGN:
            from .video_aligner import AlignmentError

            raise AlignmentError(msg)
        raise KcmcError(rc, msg)


class Context:
    """A per-device kcmc_ctx (owns the uploaded RANSAC hypothesis tables)."""

    def __init__(self, device: int):
        self.device = device
        self._h = P()
        check(load().kcmc_create(device, ctypes.byref(self._h)))

    @property
    def handle(self) -> P:
        return self._h

    def close(self) -> None:
        if self._h:
            load().kcmc_destroy(self._h)
            self._h = P()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_contexts = {}


def context(device: int) -> Context:
    with _lock:
        ctx = _contexts.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _contexts[device] = ctx
    return ctx
