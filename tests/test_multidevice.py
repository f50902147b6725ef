"""The single-process multi-device split (kcmc_amd.multidevice) on CPU: the slab partition
of a stack and the split hot path's cross-slab logic -- one vote merge over every slab,
per-slab lookup + RANSAC, one global post-processing, per-slab warps with their rows of
the global maps -- with the oracle's CPU stand-ins for the per-frame stages (test
infrastructure; tests/test_distributed.py's).  Splitting a stack into 1, 2 or 3 slabs must
not change a single value, also when the frames around a slab boundary have no model (the
NaN gap is interpolated across the boundary) and with temporal downsampling (rate 2: the
NaN padding of VA:338-344 stays inside a slab)."""
import dataclasses

import numpy as np
import pytest
import torch

from kcmc_amd import multidevice as md
from kcmc_amd import pipeline, synthetic
from test_distributed import D, HW, N_TPL, _oracle_stages


@pytest.mark.parametrize("F,rate,parts", [(10, 1, 3), (10, 3, 4), (7, 2, 8), (1, 1, 4), (12, 5, 2), (0, 1, 2)])
def test_split_frames_partition(F, rate, parts):
    rs = md.split_frames(F, rate, parts)
    n_sample = -(-F // rate)
    assert len(rs) == min(parts, n_sample)
    assert [r.s0 for r in rs] == ([0] if rs else []) + [r.s1 for r in rs[:-1]]  # contiguous sample slabs
    assert (rs[-1].s1 if rs else 0) == n_sample
    assert [r.f0 for r in rs] == ([0] if rs else []) + [r.f1 for r in rs[:-1]]  # contiguous full-rate slabs
    assert (rs[-1].f1 if rs else 0) == F
    for r in rs:
        assert r.f0 == r.s0 * rate and r.s1 > r.s0
    sizes = [r.s1 - r.s0 for r in rs]
    assert not sizes or max(sizes) - min(sizes) <= 1  # balanced
    with pytest.raises(ValueError):
        md.split_frames(F, 0, parts)


def test_slab_keypoints_cut_the_csr():
    q_off = np.array([0, 3, 3, 7, 12, 20], np.int32)
    a, b, off = md.slab_keypoints(q_off, md.SlabRange(1, 4, 1, 4))
    assert (a, b) == (3, 12) and off.tolist() == [0, 0, 4, 9]


def _stack(n_sample, rate, model, blind=()):
    """A stack of n_sample * rate frames (each with its own content) and the keypoints of
    its sample frames; sample frames in ``blind`` get descriptors unrelated to the template
    (no model: a NaN gap)."""
    ks = synthetic.make_keypoints(n_sample, N_TPL, D, HW, seed=5, frame_seed=1, model=model)
    rng = np.random.default_rng(3)
    for f in blind:
        a, b = ks.q_off[f], ks.q_off[f + 1]
        ks.des_q[a:b] = rng.integers(0, 256, (b - a, D), dtype=np.uint8)
    base = synthetic.make_texture(HW, seed=1)
    frames = np.stack([np.roll(base, (3 * f, 7 * f), axis=(0, 1)) for f in range(n_sample * rate)])
    return ks, frames


def _cpu_slabs(ks, frames, ranges):
    out = []
    for r in ranges:
        a, b, off = md.slab_keypoints(ks.q_off, r)
        out.append(pipeline.SlabInputs(torch.from_numpy(frames[r.f0:r.f1].copy()), torch.from_numpy(ks.des_tpl),
                                       torch.from_numpy(ks.kp_tpl), torch.from_numpy(ks.des_q[a:b]),
                                       torch.from_numpy(ks.kp_q[a:b]), torch.from_numpy(off), off))
    return out


@pytest.mark.parametrize("model,rate,blind", [("euclidean", 1, (4, 5, 6)), ("euclidean", 2, (0, 1, 5)),
                                              ("affine", 1, (3, 4, 5, 6, 7)), ("euclidean", 1, (8, 9))])
def test_split_equals_one_slab(model, rate, blind):
    n_sample = 10
    ks, frames = _stack(n_sample, rate, model, blind)
    cfg = pipeline.AlignConfig(n_kp_global=20, ransac_model=model, frame_downsample_rate=rate)
    st = _oracle_stages(model)
    ref = md.align_split(_cpu_slabs(ks, frames, md.split_frames(len(frames), rate, 1)),
                         md.split_frames(len(frames), rate, 1), cfg, impl=st)
    assert len(ref.skipped) >= len(blind)  # the premise: frames without a model
    # parts 1 with the warp behind the post-processing for every frame (no warp_params):
    # the device-map warp plus the re-warp of the frames without a model must equal it
    for parts, impl in ((1, dataclasses.replace(st, warp_params=None)), (2, st), (3, st), (4, st)):
        rs = md.split_frames(len(frames), rate, parts)
        got = md.align_split(_cpu_slabs(ks, frames, rs), rs, cfg, impl=impl)
        np.testing.assert_array_equal(got.affines, ref.affines)
        np.testing.assert_array_equal(got.euclidean, ref.euclidean)
        assert got.skipped == ref.skipped and got.interpolated == ref.interpolated
        np.testing.assert_array_equal(torch.cat(got.aligned).numpy(), torch.cat(ref.aligned).numpy())
        np.testing.assert_array_equal(md.gather_aligned(got), torch.cat(ref.aligned).numpy())


def test_split_rejects_mismatched_ranges():
    ks, frames = _stack(5, 1, "euclidean")
    rs = md.split_frames(5, 1, 2)
    slabs = _cpu_slabs(ks, frames, rs)
    with pytest.raises(ValueError):
        md.align_split(slabs, rs[:1], pipeline.AlignConfig(n_kp_global=20), impl=_oracle_stages())
    with pytest.raises(ValueError):
        md.align_split(slabs[::-1], rs, pipeline.AlignConfig(n_kp_global=20), impl=_oracle_stages())
