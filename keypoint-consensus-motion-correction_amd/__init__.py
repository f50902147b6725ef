"""kcmc_amd -- MI355X-native alignment hot path of keypoint-consensus motion correction.

Drop-in for the per-frame hot path of VideoAligner
(TheAustinator/keypoint-consensus-motion-correction, VideoAligner.py): descriptor
matching against the template, seeded RANSAC of the rigid frame motion and the
final warp run as hand-written HIP kernels for gfx950 (libkcmc.so, C ABI in
include/kcmc.h); the host keeps the reference's Python API.

Import as ``import kcmc_amd`` (the repository-root shim ``kcmc_amd.py`` maps that
name onto this directory).
"""
from .affines import AlignmentError
from .video_aligner import LoResVideoAligner, VideoAligner

__all__ = ["VideoAligner", "LoResVideoAligner", "AlignmentError"]
__version__ = "0.1.0"
