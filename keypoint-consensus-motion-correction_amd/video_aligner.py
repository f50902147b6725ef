"""VideoAligner with the reference's public surface, running the hot path on MI355X.

Mirror of /root/reference/VideoAligner.py (VA:15-510): same class names, class
constants, ``align_images`` signature/returns and per-frame static helpers.  The
per-frame joblib stages (VA:117-123, 137-142, 150) are replaced by one batched HIP
launch each (``pipeline.align_slab``); the helpers that the reference runs per frame
(``_get_frame_keypoints``, ``_compute_euclidean_affine``, ``_apply_affine``) run the
same kernels on a batch of one, so code written against the reference keeps working.

Differences, all deliberate:
  * Keypoint detection still needs an OpenCV-compatible detector object
    (``detectAndCompute(img, mask) -> (keypoints with .pt, uint8 descriptors)``).
    OpenCV is not part of this image; ``DETECTOR_CONSTRUCTOR_DICT`` uses cv2 when it is
    importable and accepts any registered factory.  ``align_keypoints`` is the hot-path
    entry for precomputed keypoints/descriptors.
  * numpy >= 1.24 made the reference crash on ragged per-frame point lists (VA:284-285);
    ``_lookup_consensus_kps`` returns numpy<1.24-style object arrays instead.
  * Constants are read from the instance's class, so subclass overrides take effect
    everywhere (the reference's static methods read ``VideoAligner.X``; defaults equal).
"""
from __future__ import annotations

import time
from collections import Counter
from logging import LoggerAdapter, getLogger
from multiprocessing import cpu_count
from typing import Callable, List, Optional, Sequence, Set, Tuple, Union

import numpy as np
import torch

from . import affines as _aff
from . import multidevice as _md
from . import pipeline as _pl
from . import stages
from .affines import AlignmentError


def _cv2_factory(name: str) -> Callable:
    def make():
        try:
            import cv2  # type: ignore
        except ImportError as e:  # pragma: no cover - cv2 absent in this image
            raise RuntimeError(
                f"OpenCV is not installed, so '{name}' is unavailable: register a detector factory in "
                "VideoAligner.DETECTOR_CONSTRUCTOR_DICT or call align_keypoints() with precomputed keypoints"
            ) from e
        return getattr(cv2, name)()

    make.__name__ = name
    return make


class _CvKeyPoint:
    __slots__ = ("pt",)

    def __init__(self, x: float, y: float):
        self.pt = (x, y)


class GpuOrbDetector:
    """The build's ORB-style detector (csrc/orb.hip) behind the OpenCV
    detector interface the reference uses (VA:114-116, VA:190-192):
    ``detectAndCompute(img_u8, mask) -> (keypoints with .pt, uint8 [n, 32] descriptors)``.
    ``align_images`` recognises it and detects on the whole device-resident stack at once."""

    def __init__(self, params=None):
        from . import orb

        self.params = params or orb.OrbParams()

    def detectAndCompute(self, image, mask=None):  # noqa: N802 (OpenCV's name)
        if mask is not None:
            raise NotImplementedError("detection masks are not supported by the GPU detector")
        dev = torch.device("cuda", torch.cuda.current_device())
        img = image if isinstance(image, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        k = stages.detect_orb(img.to(dev).reshape(1, *img.shape[-2:]).contiguous(), self.params)
        n = int(k.count.cpu()[0])
        kp = k.kp[0, :n].cpu().numpy()
        return [_CvKeyPoint(float(x), float(y)) for x, y in kp], k.des[0, :n].cpu().numpy()


def _as_numpy(x) -> np.ndarray:
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


class VideoAligner:
    AlignmentError = AlignmentError

    FRAME_SAMPLE_RATE = 100  # Hz
    SPATIAL_DOWNSAMPLE_RATE = 1
    N_JOBS_PARALLEL = cpu_count()
    DETECTOR_CONSTRUCTOR_DICT = {
        "akaze": _cv2_factory("AKAZE_create"),
        "brisk": _cv2_factory("BRISK_create"),
        # New: the build's exact ORB-style detector on the GPU (no OpenCV needed).
        "orb": GpuOrbDetector,
    }
    N_KP_GLOBAL_MIN = 5
    N_KP_FRAME_SKIP = 3
    TEMPLATE_FRAME_LOC = 0.5
    MAX_FRAC_INTERPOLATED = 0.2
    DESCRIPTOR_DISTANCE_RATIO_THRESH = 0.75
    MEDIAN_KEYPOINT_INLIER_DISTANCE_RANGE = (0.5, 2.0)
    IMAGE_NORM_MAX_PERCENTILE = 99.99
    MAX_PIXEL_UINT8 = 255
    RANSAC_MIN_SAMPLES = 2
    RANSAC_RESIDUAL_THRESH = 2
    RANSAC_MAX_TRIALS = 1000
    RANDOM_SEED = 42
    # New: the GPUs align_images / align_keypoints spread the frames over, as the
    # reference's _parallelize spreads them over every core (VA:21, VA:460-471): None = every
    # visible device (the current one first; one contiguous frame slab per device, the
    # cross-frame consensus and gap interpolation made once on the host, kcmc_amd.multidevice);
    # a list pins them (a device may repeat: two slabs on one GPU).
    DEVICES: Optional[Sequence[int]] = None
    # New: one GPU for everything (used when DEVICES is None; None = as DEVICES).  The
    # per-frame helpers (_get_frame_keypoints, _compute_euclidean_affine, _apply_affine)
    # run on the first device.
    DEVICE: Optional[int] = None
    # New (extension, BASELINE configs 3-5): the skimage model class RANSAC fits --
    # "euclidean" (the reference's EuclideanTransform, VA:311), "affine"
    # (AffineTransform, min_samples 3) or "projective" (ProjectiveTransform, min_samples 4,
    # frames warped with warpPerspective).
    RANSAC_MODEL = "euclidean"
    # New (opt-in, not the reference's matcher): the BFMatcher norm -- "l2" (the
    # reference's cv2.BFMatcher() default, VA:194) or "hamming" (NORM_HAMMING, for binary
    # ORB/BRIEF/AKAZE descriptors; csrc/match_hamming.hip).
    MATCH_NORM = "l2"

    def __init__(self, logger: LoggerAdapter = None):
        self.logger = logger
        if self.logger is None:
            self.logger = getLogger(self.__class__.__name__)
        self.affines = None
        self.aligned_imgs = None
        self.interpolated_idxs = None
        self._kp_template = None
        self._des_template = None

    # ------------------------------------------------------------------ helpers
    @classmethod
    def _devices(cls) -> List[int]:
        """The devices of the hot path: DEVICES, else [DEVICE], else every visible device
        with the current one first."""
        if not torch.cuda.is_available():
            from ._lib import KcmcLibraryError

            raise KcmcLibraryError("no GPU visible: the kcmc hot path runs on MI355X only (no CPU fallback)")
        if cls.DEVICES is not None:
            devs = [int(d) for d in cls.DEVICES]
            if not devs:
                raise ValueError("VideoAligner.DEVICES is empty")
            return devs
        if cls.DEVICE is not None:
            return [int(cls.DEVICE)]
        cur = torch.cuda.current_device()
        return [cur] + [d for d in _md.visible_devices() if d != cur]

    @classmethod
    def _device(cls) -> torch.device:
        return torch.device("cuda", cls._devices()[0])

    def _config(self, n_kp_global: int, frame_downsample_rate: int = 1) -> _pl.AlignConfig:
        cls = type(self)
        d_lo, d_hi = (0.5, 2)  # hard-coded at VA:209 (MEDIAN_KEYPOINT_INLIER_DISTANCE_RANGE is unused there)
        return _pl.AlignConfig(
            n_kp_global=int(n_kp_global), n_kp_global_min=cls.N_KP_GLOBAL_MIN, n_kp_frame_skip=cls.N_KP_FRAME_SKIP,
            ratio=cls.DESCRIPTOR_DISTANCE_RATIO_THRESH, d_lo=d_lo, d_hi=d_hi, ransac_trials=cls.RANSAC_MAX_TRIALS,
            ransac_threshold=float(cls.RANSAC_RESIDUAL_THRESH), ransac_min_samples=cls.RANSAC_MIN_SAMPLES,
            seed=cls.RANDOM_SEED, spatial_rate=cls.SPATIAL_DOWNSAMPLE_RATE,
            frame_downsample_rate=int(frame_downsample_rate), ransac_model=cls.RANSAC_MODEL,
            match_norm=cls.MATCH_NORM)

    # ------------------------------------------------------------- public API
    def align_images(
        self,
        images: np.ndarray,
        n_kp_global: int,
        detector_algorithm: str,
        frame_rate: int,
        masked_template: Optional[np.ndarray] = None,
        patch: Optional[Tuple[float, float, float, float]] = None,
    ) -> Tuple[np.ndarray, np.ndarray, List[int]]:
        """Register a uint16 stack [frames, x, y] to a template frame (VA:57-158).

        Returns (aligned_imgs, euclidean_transforms [n, 3] = (tx, ty, rotation),
        skipped_idxs).  A device tensor input yields a device tensor output.
        """
        self.logger.info(f"aligning {len(images)} frames with n_kp_global: {n_kp_global} and {detector_algorithm}")
        if not 0 <= self.TEMPLATE_FRAME_LOC <= 1:
            raise ValueError("`template_frame_loc` must be between 0 and 1")
        on_device = isinstance(images, torch.Tensor)
        images_np = None if on_device else np.asarray(images)
        if masked_template is not None:
            template = _as_numpy(masked_template)
        else:
            template_idx = int(len(images) * self.TEMPLATE_FRAME_LOC)
            template = _as_numpy(images[template_idx])
            self.logger.info(f"no masked template provided. Using frame {template_idx} as template")

        frame_downsample_rate = max(1, frame_rate // self.FRAME_SAMPLE_RATE)
        devices = self._devices()
        ranges = _md.split_frames(len(images), frame_downsample_rate, len(devices))
        if len(ranges) > 1:
            return self._align_images_split(images, template, n_kp_global, detector_algorithm, frame_downsample_rate,
                                            patch, devices[:len(ranges)], ranges)

        self.logger.info("normalizing frames...")
        t_start = time.time()
        # VA:100-108 on the device: the stack is uploaded once (and reused by the warp),
        # percentile and max-scaling run as HIP kernels; the uint8 copy comes back for the
        # host detector.
        assert (images.dtype == torch.uint16) if on_device else (images_np.dtype == np.uint16)  # VA:104
        dev = self._device()
        frames = images if on_device else torch.from_numpy(np.ascontiguousarray(images_np)).to(dev)
        brightest_px = self._get_brightest_px(frames)
        u8_dev = self._max_scale_images(frames, None, brightest_px, np.uint8)[0]
        _, template_i8 = self._max_scale_images(None, template, brightest_px, np.uint8)
        detector = self.DETECTOR_CONSTRUCTOR_DICT[detector_algorithm]()
        on_gpu = isinstance(detector, GpuOrbDetector) and frames.dim() == 3
        if not on_gpu:
            images_i8 = u8_dev.cpu().numpy()
            images_sample, template = self._downsample(images_i8, template_i8, frame_downsample_rate,
                                                       self.SPATIAL_DOWNSAMPLE_RATE)
        self.logger.info(f"normalized frames in: {round(time.time() - t_start)} s")

        self.logger.info("identifying keypoints...")
        t_start = time.time()
        if on_gpu:  # f1: detection of the whole stack on the device (f4: downsample there too)
            sample_dev, tpl_dev = _pl.downsample_u8(u8_dev, torch.from_numpy(np.ascontiguousarray(template_i8)).to(dev)[None],
                                                    frame_downsample_rate, self.SPATIAL_DOWNSAMPLE_RATE)
            kt = stages.detect_orb(tpl_dev, detector.params)
            kq = stages.detect_orb(sample_dev, detector.params)
            n_t = int(kt.count.cpu()[0])
            self._kp_template = kt.kp[0, :n_t].cpu().numpy()
            self._des_template = kt.des[0, :n_t].cpu().numpy()
            kp_q, des_q, q_off, q_off_host = stages.keypoints_csr(kq)
            inp = _pl.SlabInputs(frames, kt.des[0, :n_t].contiguous(), kt.kp[0, :n_t].contiguous(), des_q, kp_q,
                                 q_off, q_off_host)
            self.logger.info(f"identified keypoints in: {round(time.time() - t_start)} s")
            aligned, eu, skipped = self._align_inputs(inp, n_kp_global, frame_downsample_rate, patch)
            return (aligned if on_device else aligned.cpu().numpy()), eu, skipped
        kp_t, des_t = detector.detectAndCompute(template, None)
        self._kp_template = np.array([p.pt for p in kp_t])
        self._des_template = des_t
        kp_list, des_list = [], []
        for img in images_sample:
            kq, dq = detector.detectAndCompute(img, None)
            kp_list.append(np.array([p.pt for p in kq], dtype=np.float64).reshape(-1, 2))
            des_list.append(np.asarray(dq, dtype=np.uint8).reshape(len(kq), -1))
        self.logger.info(f"identified keypoints in: {round(time.time() - t_start)} s")
        aligned, eu, skipped = self._align_detected(frames, self._kp_template, self._des_template, kp_list, des_list,
                                                    n_kp_global, frame_downsample_rate, patch)
        if not on_device:
            aligned = aligned.cpu().numpy()
        return aligned, eu, skipped

    def _align_images_split(self, images, template, n_kp_global, detector_algorithm, rate, patch, devices, ranges):
        """align_images with the stack split over several devices (kcmc_amd.multidevice):
        each slab's frames uploaded to its device, the 99.99th percentile of the whole stack
        from the summed per-device histograms, max-scaling and (GPU detector) detection per
        device, then the split hot path."""
        on_device = isinstance(images, torch.Tensor)
        self.logger.info("normalizing frames...")
        t_start = time.time()
        assert (images.dtype == torch.uint16) if on_device else (np.asarray(images).dtype == np.uint16)  # VA:104
        parts = _md.split_to_devices(images if on_device else np.asarray(images), ranges, devices)
        brightest_px = stages.brightest_px(parts, self.IMAGE_NORM_MAX_PERCENTILE)
        u8_parts = []
        for p in parts:  # each slab's work under its own device (launches, workspaces, allocations)
            with _md._on(p):
                u8_parts.append(self._max_scale_images(p, None, brightest_px, np.uint8)[0])
        _, template_i8 = self._max_scale_images(None, template, brightest_px, np.uint8)
        detector = self.DETECTOR_CONSTRUCTOR_DICT[detector_algorithm]()
        on_gpu = isinstance(detector, GpuOrbDetector) and parts[0].dim() == 3
        self.logger.info(f"normalized frames in: {round(time.time() - t_start)} s")

        self.logger.info("identifying keypoints...")
        t_start = time.time()
        cfg = self._config(n_kp_global, rate)
        if on_gpu:  # f1 per device: each slab's sample frames detected where they live
            tpl_u8 = np.ascontiguousarray(template_i8)
            samples = []
            for u in u8_parts:
                with _md._on(u):
                    samples.append(_pl.downsample_u8(u, torch.from_numpy(tpl_u8).to(u.device)[None], rate,
                                                     self.SPATIAL_DOWNSAMPLE_RATE))
            with _md._on(samples[0][1]):
                kt = stages.detect_orb(samples[0][1], detector.params)
            n_t = int(kt.count.cpu()[0])
            self._kp_template = kt.kp[0, :n_t].cpu().numpy()
            self._des_template = kt.des[0, :n_t].cpu().numpy()
            slabs = []
            for fr, (smp, _) in zip(parts, samples):
                with _md._on(smp):
                    kp_q, des_q, q_off, q_off_host = stages.keypoints_csr(stages.detect_orb(smp, detector.params))
                dev = fr.device
                slabs.append(_pl.SlabInputs(fr, torch.from_numpy(self._des_template).to(dev),
                                            torch.from_numpy(self._kp_template).to(dev), des_q, kp_q, q_off, q_off_host))
        else:
            images_i8 = np.concatenate([u.cpu().numpy() for u in u8_parts])
            images_sample, template = self._downsample(images_i8, template_i8, rate, self.SPATIAL_DOWNSAMPLE_RATE)
            kp_t, des_t = detector.detectAndCompute(template, None)
            self._kp_template = np.array([p.pt for p in kp_t])
            self._des_template = des_t
            kp_list, des_list = [], []
            for img in images_sample:
                kq, dq = detector.detectAndCompute(img, None)
                kp_list.append(np.array([p.pt for p in kq], dtype=np.float64).reshape(-1, 2))
                des_list.append(np.asarray(dq, dtype=np.uint8).reshape(len(kq), -1))
            kp_flat, des_flat, q_off = self._csr(kp_list, des_list, np.asarray(des_t).shape[1])
            slabs = _md.make_slabs(parts, ranges, np.asarray(des_t, np.uint8), self._kp_template, kp_flat, des_flat,
                                   q_off)
        self.logger.info(f"identified keypoints in: {round(time.time() - t_start)} s")
        return self._finish_split(slabs, ranges, cfg, patch, images.device if on_device else None)

    def _finish_split(self, slabs, ranges, cfg, patch, out_device):
        self.logger.info("generating keypoint consensus...")
        t_start = time.time()
        res = _md.align_split(slabs, ranges, cfg, logger=self.logger)
        self.interpolated_idxs = res.interpolated
        self.logger.info(f"aligned frames in: {round(time.time() - t_start)} s")
        aligned = _md.gather_aligned(res, out_device)
        if patch is not None:
            x_start, y_start, width, height = patch
            aligned = aligned[:, x_start:x_start + width, y_start:y_start + height]
        return aligned, res.euclidean, res.skipped

    @staticmethod
    def _csr(kp_list, des_list, D):
        q_off = np.zeros(len(kp_list) + 1, np.int32)
        q_off[1:] = np.cumsum([len(k) for k in kp_list])
        kp_flat = np.concatenate(kp_list).astype(np.float64) if q_off[-1] else np.zeros((0, 2))
        des_flat = np.concatenate(des_list).astype(np.uint8) if q_off[-1] else np.zeros((0, D), np.uint8)
        return kp_flat, des_flat, q_off

    def align_keypoints(
        self,
        images,
        kp_template: np.ndarray,
        des_template: np.ndarray,
        kp_query: Sequence[np.ndarray],
        des_query: Sequence[np.ndarray],
        n_kp_global: int,
        frame_rate: int = 30,
        patch: Optional[Tuple[float, float, float, float]] = None,
    ):
        """The hot path with precomputed keypoints: per SAMPLE frame
        (images[::max(1, frame_rate // FRAME_SAMPLE_RATE)]) keypoint coordinates [n, 2]
        and uint8 descriptors [n, D]; template keypoints/descriptors likewise."""
        self._kp_template = np.asarray(kp_template, dtype=np.float64).reshape(-1, 2)
        self._des_template = np.asarray(des_template, dtype=np.uint8)
        rate = max(1, frame_rate // self.FRAME_SAMPLE_RATE)
        return self._align_detected(images, self._kp_template, self._des_template, list(kp_query), list(des_query),
                                    n_kp_global, rate, patch)

    def _align_detected(self, images, kp_template, des_template, kp_list, des_list, n_kp_global, rate, patch):
        to_host = not isinstance(images, torch.Tensor)
        kp_flat, des_flat, q_off = self._csr(kp_list, des_list, des_template.shape[1])
        devices = self._devices()
        ranges = _md.split_frames(len(images), rate, len(devices))
        if len(ranges) > 1:  # every device its slab of frames (kcmc_amd.multidevice)
            parts = _md.split_to_devices(images if not to_host else np.asarray(images), ranges, devices)
            slabs = _md.make_slabs(parts, ranges, des_template, kp_template, kp_flat, des_flat, q_off)
            return self._finish_split(slabs, ranges, self._config(n_kp_global, rate), patch,
                                      None if to_host else images.device)
        dev = torch.device("cuda", devices[0])
        frames = torch.from_numpy(np.ascontiguousarray(images)).to(dev) if to_host else images.contiguous()
        inp = _pl.SlabInputs(
            frames=frames,
            des_tpl=torch.from_numpy(np.ascontiguousarray(des_template, np.uint8)).to(dev),
            kp_tpl=torch.from_numpy(np.ascontiguousarray(kp_template, np.float64)).to(dev),
            des_q=torch.from_numpy(np.ascontiguousarray(des_flat)).to(dev),
            kp_q=torch.from_numpy(np.ascontiguousarray(kp_flat).reshape(-1, 2)).to(dev),
            q_off=torch.from_numpy(q_off).to(dev),
            q_off_host=q_off,
        )
        return self._align_inputs(inp, n_kp_global, rate, patch, to_host=to_host)

    def _align_inputs(self, inp, n_kp_global, rate, patch, to_host: bool = False):
        cfg = self._config(n_kp_global, rate)
        self.logger.info("generating keypoint consensus...")
        t_start = time.time()
        res = _pl.align_slab(inp, cfg, logger=self.logger)
        self.interpolated_idxs = res.interpolated
        self.logger.info(f"aligned frames in: {round(time.time() - t_start)} s")
        aligned = res.aligned
        if patch is not None:
            x_start, y_start, width, height = patch
            x_end = x_start + width
            y_end = y_start + height
            aligned = aligned[:, x_start:x_end, y_start:y_end]
        if to_host:
            aligned = aligned.cpu().numpy()
        return aligned, res.euclidean, res.skipped

    # ------------------------------------------------ per-frame helpers (VA:160-458)
    @classmethod
    def _get_frame_keypoints(cls, i: int, image: np.ndarray, kp_template: np.ndarray, des_template: np.ndarray,
                             detector_algorithm: str) -> Tuple[Set[int], np.ndarray, str]:
        """VA:160-222 for one frame (detection on the host, matching on the GPU)."""
        detector = cls.DETECTOR_CONSTRUCTOR_DICT[detector_algorithm]()
        kq, dq = detector.detectAndCompute(image, None)
        kp_query = np.array([p.pt for p in kq], dtype=np.float64).reshape(-1, 2)
        return cls._match_frame(i, kp_query, np.asarray(dq, np.uint8), kp_template, des_template)

    @classmethod
    def _match_frame(cls, i, kp_query, des_query, kp_template, des_template):
        dev = cls._device()
        q_off = np.array([0, len(kp_query)], np.int32)
        m = stages.match_frames(
            torch.from_numpy(np.ascontiguousarray(des_template, np.uint8)).to(dev),
            torch.from_numpy(np.ascontiguousarray(kp_template, np.float64)).to(dev),
            torch.from_numpy(np.ascontiguousarray(des_query, np.uint8)).to(dev),
            torch.from_numpy(np.ascontiguousarray(kp_query, np.float64)).to(dev),
            torch.from_numpy(q_off).to(dev), q_off, ratio=cls.DESCRIPTOR_DISTANCE_RATIO_THRESH)
        n_tpl = len(kp_template)
        bits = m.keep_bits.cpu().numpy().view(np.uint32)[0]
        kept = [k for k in range(n_tpl) if (bits[k >> 5] >> (k & 31)) & 1]
        c = m.counts.cpu().numpy()[0]
        log_str = (
            f"frame {i}:\n"
            f"\t{int(c[0])} unfiltered features identified\n"
            f"\t{int(c[1])} matches identified between frame and template\n"
            f"\t{int(c[2])} matches after feature-space ratio filter\n"
            f"\t{int(c[3])} matches after distance-based outlier rejection"
        )
        return set(kept), m.kp_ordered.cpu().numpy()[0], log_str

    def _get_consensus_kps(self, kp_idxs_list: List[set], n_frames: int, n_kp_global: int) -> Set[int]:
        """VA:224-249: the n_kp_global most frequently matched template keypoints."""
        counts = Counter([x for s in kp_idxs_list for x in s])
        votes = [x for x in counts.most_common(n_kp_global)]
        if len(votes) < self.N_KP_GLOBAL_MIN:
            raise VideoAligner.AlignmentError(
                "Too few keypoints found. Try a higher quality video, or decrease `VideoAligner.N_KP_GLOBAL_MIN`")
        consensus_idxs, vote_match_rates = zip(*votes)
        vote_match_rates = np.array(vote_match_rates) / n_frames
        self.logger.info(f"top n keypoints match rates: {vote_match_rates}")
        return set(consensus_idxs)

    def _lookup_consensus_kps(self, consensus_idxs: Set[int], kp_idxs_list: List[Set[int]],
                              kp_query_list: List[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
        """VA:251-286 (object arrays for ragged frames, as numpy < 1.24 produced)."""
        tk, qk = [], []
        for i in range(len(kp_query_list)):
            idx = list(consensus_idxs.intersection(kp_idxs_list[i]))
            tk.append(self._kp_template[idx])
            qk.append(np.asarray(kp_query_list[i])[idx])
            if len(qk[-1]) < self.N_KP_FRAME_SKIP:
                self.logger.info(
                    f"transform for frame {i} not estimated due to low keypoint count: "
                    f"({len(qk[-1])}). Will be interpolated based on other frames instead")

        def arr(lst):
            try:
                return np.array(lst)
            except ValueError:
                out = np.empty(len(lst), dtype=object)
                for k, v in enumerate(lst):
                    out[k] = v
                return out

        return arr(tk), arr(qk)

    @classmethod
    def _compute_euclidean_affine(cls, kp_template: np.ndarray, kp_query: np.ndarray,
                                  spatial_downsample_rate: Union[float, int]) -> Optional[np.ndarray]:
        """VA:288-323 for one frame: seeded rigid RANSAC on the GPU (NaN on failure)."""
        kp_query = np.asarray(kp_query, dtype=np.float64).reshape(-1, 2)
        kp_template = np.asarray(kp_template, dtype=np.float64).reshape(-1, 2)
        if len(kp_query) < cls.N_KP_FRAME_SKIP:
            return np.full((2, 3), np.nan)
        dev = cls._device()
        off = np.array([0, len(kp_query)], np.int32)
        r = stages.ransac_rigid(
            torch.from_numpy(np.ascontiguousarray(kp_query)).to(dev),
            torch.from_numpy(np.ascontiguousarray(kp_template)).to(dev),
            torch.from_numpy(off).to(dev), off, trials=cls.RANSAC_MAX_TRIALS,
            residual_threshold=float(cls.RANSAC_RESIDUAL_THRESH), spatial_rate=spatial_downsample_rate,
            n_skip=cls.N_KP_FRAME_SKIP, seed=cls.RANDOM_SEED, min_samples=cls.RANSAC_MIN_SAMPLES)
        return r.params.cpu().numpy()[0]

    _process_affines = staticmethod(_aff.process_affines)
    _interpolate_affines = staticmethod(_aff.interpolate_affines)
    _get_euclidean_transforms = staticmethod(_aff.euclidean_transforms)

    @staticmethod
    def _interpolate_affines_frame_range(base_affines: np.ndarray, failed_idx_range: range) -> List[np.ndarray]:
        """VA:409-437."""
        xs = np.arange(failed_idx_range[0], failed_idx_range[-1] + 1)
        out = _aff._lerp_gap(base_affines[0], base_affines[1], failed_idx_range[0] - 1, failed_idx_range[-1] + 1, xs)
        return [a for a in out]

    @classmethod
    def _apply_affine(cls, image: np.ndarray, affine: np.ndarray) -> np.ndarray:
        """VA:455-458: cv2.warpAffine(image, affine, (W, H), INTER_LINEAR) on the GPU."""
        dev = cls._device()
        img = torch.from_numpy(np.ascontiguousarray(image, np.uint16)[None]).to(dev)
        a = torch.from_numpy(np.ascontiguousarray(affine, np.float64).reshape(1, 2, 3)).to(dev)
        return stages.warp_affine_u16(img, a).cpu().numpy()[0]

    def _parallelize(self, func: Callable, *sequences: Sequence, **kwargs) -> List:
        """VA:460-465: func over the equal-length sequences, results in order, in a joblib
        process pool of N_JOBS_PARALLEL workers (backend "multiprocessing", as the reference)
        -- for a subclass's own (picklable, CPU) per-frame function.  This package's functions
        run in this process instead: they are GPU-backed, a forked worker cannot use the
        parent's GPU context, and the hot path batches them anyway."""
        r = range(len(sequences[0]))
        mod = getattr(func, "__module__", "") or ""
        if mod.split(".")[0] == __name__.split(".")[0] or int(self.N_JOBS_PARALLEL) <= 1 or len(r) <= 1:
            return [func(*[x[i] for x in sequences], **kwargs) for i in r]
        from joblib import Parallel, delayed

        with Parallel(n_jobs=int(self.N_JOBS_PARALLEL), backend="multiprocessing") as parallel:
            return list(parallel(delayed(func)(*[x[i] for x in sequences], **kwargs) for i in r))

    def _parallelize_i(self, func: Callable, *sequences: Sequence, **kwargs) -> List:
        r = range(len(sequences[0]))
        return self._parallelize(func, r, *sequences, **kwargs)

    @staticmethod
    def _convert_to_array(*args: Sequence):
        return tuple(np.array(arg) for arg in args)

    @classmethod
    def _get_brightest_px(cls, images) -> Union[float, int]:
        """VA:479-482: np.percentile(images, 99.99).  A uint16 device tensor takes the exact
        HIP path (two histogram passes + numpy's interpolation); a host array is the
        reference's own numpy call."""
        if isinstance(images, torch.Tensor):
            return stages.brightest_px(images.contiguous(), cls.IMAGE_NORM_MAX_PERCENTILE)
        return np.percentile(images, cls.IMAGE_NORM_MAX_PERCENTILE)

    @classmethod
    def _max_scale_images(cls, images, template, brightest_px: float, output_dtype: type):
        """VA:484-492.  uint16 device tensors are scaled on the GPU through the table of
        the reference's expression (bit-exact); host arrays use the expression itself.
        Either argument may be None (returned as None)."""
        max_px = cls.MAX_PIXEL_UINT8

        def scale(x):
            if x is None:
                return None
            if isinstance(x, torch.Tensor) and x.dtype == torch.uint16 and output_dtype == np.uint8:
                return stages.max_scale_u8(x.contiguous(), brightest_px, max_px=max_px)
            x = _as_numpy(x)
            if x.dtype == np.uint16 and output_dtype == np.uint8:
                return stages.max_scale_lut(brightest_px, max_px)[x]
            return np.clip(x / brightest_px * max_px, a_min=0, a_max=max_px).astype(output_dtype)

        return scale(images), scale(template)

    @staticmethod
    def _downsample(images: np.ndarray, template: np.ndarray, frame_downsample_rate: int,
                    spatial_downsample_rate: Union[float, int]) -> Tuple[np.ndarray, np.ndarray]:
        """VA:494-506: every rate-th frame and, when the rate is not 1, cv2.pyrDown of the
        sample frames and the template -- here the device kernel (stages.pyr_down_u8, via
        pipeline.downsample_u8) with the reference's dstsize quirk kept."""
        if int(frame_downsample_rate) == 1:
            return images[::1], template
        dev = VideoAligner._device()
        f = torch.from_numpy(np.ascontiguousarray(images, np.uint8)).to(dev)
        t = torch.from_numpy(np.ascontiguousarray(template, np.uint8)).to(dev)[None]
        s, t = _pl.downsample_u8(f, t, frame_downsample_rate, spatial_downsample_rate)
        return s.cpu().numpy(), t[0].cpu().numpy()


class LoResVideoAligner(VideoAligner):
    SPATIAL_DOWNSAMPLE_RATE = 2
