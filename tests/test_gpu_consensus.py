"""The device consensus (csrc/consensus.hip) against the native host consensus, which is
itself pinned to live CPython set / Counter behaviour (tests/test_host.py):

  * kcmc_consensus_vote: counts and first-occurrence keys (frame, CPython set-table slot)
    equal kcmc_consensus_vote_host bit for bit -- dense frames (ascending sets), sparse
    frames with large template indices (the slot comes from the set-insertion replay),
    empty frames, n_tpl up to 4096, thousands of frames;
  * kcmc_consensus_lookup: every frame's list(consensus & frame_set) (VA:274) equals
    kcmc_consensus_lookup_host -- both set_intersection branches (frame larger / not larger
    than the consensus), replayed and ascending results, consensus sizes 1 ... 500;
  * kcmc_params_boundary: first / last frame without NaN and their parameters."""
import numpy as np
import pytest
import torch

from kcmc_amd import stages

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _random_bits(rng, F, n_tpl, density):
    words = (n_tpl + 31) // 32
    p = rng.uniform(0, 1, n_tpl) * density
    on = np.zeros((F, words * 32), bool)
    on[:, :n_tpl] = rng.random((F, n_tpl)) < p
    return np.ascontiguousarray(np.packbits(on, axis=1, bitorder="little")).view(np.uint32)


CASES = [(1, 8, 0.5), (3, 33, 0.9), (40, 100, 0.3), (500, 500, 0.7), (2500, 500, 0.6), (64, 500, 0.02),
         (300, 4096, 0.01), (625, 4096, 0.5), (200, 1000, 0.005), (17, 4096, 0.9), (3000, 160, 0.2)]


@pytest.mark.parametrize("F,n_tpl,density", CASES)
def test_device_vote_equals_host(dev, F, n_tpl, density):
    rng = np.random.default_rng(F * 7 + n_tpl)
    kb = _random_bits(rng, F, n_tpl, density)
    if F > 4:
        kb[F // 2] = 0  # an empty frame
    for base in (0, 12345):
        got = stages.consensus_vote(torch.from_numpy(kb.view(np.int32)).to(dev), n_tpl, base).cpu().numpy()
        exp = stages.consensus_vote_host(kb, n_tpl, base)
        np.testing.assert_array_equal(got, exp)


def test_device_vote_replays_sparse_first_frames(dev):
    """First frames whose set table is smaller than their largest key: slots from the
    replay, in many distinct first frames at once (more than the 64 replay lanes)."""
    rng = np.random.default_rng(3)
    n_tpl, F = 4096, 400
    kb = np.zeros((F, n_tpl // 32), np.uint32)
    for f in range(F):
        for t in rng.choice(n_tpl, int(rng.integers(1, 60)), replace=False):
            kb[f, t >> 5] |= np.uint32(1 << (t & 31))
    got = stages.consensus_vote(torch.from_numpy(kb.view(np.int32)).to(dev), n_tpl, 7).cpu().numpy()
    np.testing.assert_array_equal(got, stages.consensus_vote_host(kb, n_tpl, 7))


@pytest.mark.parametrize("F,n_tpl,density", CASES)
@pytest.mark.parametrize("n_kp_global", [1, 5, 50, 100, 200, 500])
def test_device_lookup_equals_host(dev, F, n_tpl, density, n_kp_global):
    rng = np.random.default_rng(F + n_tpl + n_kp_global)
    kb = _random_bits(rng, F, n_tpl, density)
    v = stages.consensus_vote_host(kb, n_tpl)
    try:
        choice = stages.consensus_merge(v, n_tpl, n_kp_global, 1)
    except BaseException:  # nothing voted
        return
    pack = torch.from_numpy(choice.pack).to(dev)
    po, pi = stages.consensus_lookup(torch.from_numpy(kb.view(np.int32)).to(dev), n_tpl, pack, choice.nc)
    po, pi = po.cpu().numpy(), pi.cpu().numpy()
    eo, ei = stages.consensus_lookup_host(kb, n_tpl, choice.cons_iter)
    np.testing.assert_array_equal(po, eo)
    np.testing.assert_array_equal(pi[: po[-1]], ei)


def test_device_lookup_frame_set_branch(dev):
    """Frames with no more keys than the consensus: set_intersection iterates the frame's
    own set, whose table order is not ascending when its keys are large (replay of the
    frame set, then of the result)."""
    rng = np.random.default_rng(8)
    n_tpl, F = 4096, 300
    kb = np.zeros((F, n_tpl // 32), np.uint32)
    common = rng.choice(n_tpl, 300, replace=False)
    for f in range(F):
        k = int(rng.integers(1, 300)) if f % 3 else 300
        for t in (common[:k] if f % 5 else rng.choice(common, k, replace=False)):
            kb[f, t >> 5] |= np.uint32(1 << (t & 31))
    v = stages.consensus_vote_host(kb, n_tpl)
    for nkg in (40, 200, 300):
        choice = stages.consensus_merge(v, n_tpl, nkg, 1)
        po, pi = stages.consensus_lookup(torch.from_numpy(kb.view(np.int32)).to(dev), n_tpl,
                                         torch.from_numpy(choice.pack).to(dev), choice.nc)
        eo, ei = stages.consensus_lookup_host(kb, n_tpl, choice.cons_iter)
        np.testing.assert_array_equal(po.cpu().numpy(), eo)
        np.testing.assert_array_equal(pi.cpu().numpy()[: eo[-1]], ei)


@pytest.mark.parametrize("shape", [(2, 3), (3, 3)])
def test_params_boundary(dev, shape):
    rng = np.random.default_rng(1)
    for F, miss in ((1, []), (5, [0, 4]), (9, list(range(9))), (700, list(range(0, 700, 3)) + [1, 698])):
        p = rng.normal(size=(F,) + shape)
        for f in miss:
            p[f, int(rng.integers(0, shape[0])), int(rng.integers(0, 3))] = np.nan
        got = stages.params_boundary(torch.from_numpy(p).to(dev)).cpu().numpy()
        ok = np.flatnonzero(~np.isnan(p.reshape(F, -1)).any(axis=1))
        E = p[0].size
        if ok.size == 0:
            assert got[0] == -1 and got[1] == -1 and np.isnan(got[2:]).all()
        else:
            assert got[0] == ok[0] and got[1] == ok[-1]
            np.testing.assert_array_equal(got[2:2 + E], p[ok[0]].ravel())
            np.testing.assert_array_equal(got[2 + E:], p[ok[-1]].ravel())
