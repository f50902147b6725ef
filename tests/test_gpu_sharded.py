"""The product's frame-sharded path on the GPU: two ranks (gloo, both on cuda:0, started
as fresh child processes) run `distributed.align_sharded` with the HIP stages and the
pipelined `OverlappedSlabs(counts=...)` on uneven slabs, with the template broadcast
from rank 0 (VA:117-123 / VA:460-465 pickle it to every worker).  The concatenated
per-rank results must be bit-identical to one single-device `align_slab` over all
frames: the vote all-gather + per-rank device lookup (VA:224-286) and the slab-boundary
all-gather + per-rank gap filling (VA:347-407) may not change a single pixel.  In the
"blind" case rank 1's frames carry random descriptors, so none of them gets a model and
the NaN gap spans rank 1's whole slab (filled from rank 0's last and rank 2's first model).

The ranks are separate interpreters (this file run as a script), launched before this
process touches the GPU in the test body."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from kcmc_amd import pipeline, synthetic  # noqa: E402

COUNTS = {2: (9, 14), 3: (9, 7, 11)}  # uneven slabs (frames per rank)
N_TPL, D, HW = 160, 32, (120, 200)
N_KP_GLOBAL = 40


def _keypoints(rank: int, slab: int, model: str, world: int = 2, blind: bool = False):
    ks = synthetic.make_keypoints(COUNTS[world][rank], N_TPL, D, HW, seed=17, frame_seed=100 * slab + rank, model=model)
    if blind and rank == 1:  # descriptors unrelated to the template: no frame of this rank gets a model
        ks.des_q[:] = np.random.default_rng(99 + slab).integers(0, 256, ks.des_q.shape, dtype=np.uint8)
    return ks


def _frames(n: int, f0: int = 0):
    """Frames f0 .. f0 + n - 1 of the job, each with its own content (global index f)."""
    base = synthetic.make_texture(HW, seed=4)
    return np.ascontiguousarray(np.stack([np.roll(base, (5 * f, 11 * f), axis=(0, 1)) for f in range(f0, f0 + n)]))


def _inputs(ks_list, dev, f0: int = 0):
    """SlabInputs of the concatenation of several ranks' keypoint sets."""
    des_q = np.concatenate([k.des_q for k in ks_list])
    kp_q = np.concatenate([k.kp_q for k in ks_list])
    off = [0]
    for k in ks_list:
        off.extend((off[-1] + k.q_off[1:]).tolist())
    q_off = np.asarray(off, np.int32)
    n = len(q_off) - 1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return pipeline.SlabInputs(t(_frames(n, f0)), t(ks_list[0].des_tpl), t(ks_list[0].kp_tpl), t(des_q), t(kp_q),
                               t(q_off), q_off)


def _rank_main(rank: int, port: int, out_dir: str, model: str, world: int, blind: bool,
               beside: bool = False) -> None:
    import torch.distributed as dist

    from kcmc_amd import distributed as kdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = pipeline.AlignConfig(n_kp_global=N_KP_GLOBAL, ransac_model=model)
    f0 = sum(COUNTS[world][:rank])
    slabs = [_inputs([_keypoints(rank, s, model, world, blind)], dev, f0) for s in range(3)]
    for inp in slabs:
        if rank != 0:  # only rank 0 holds the template; the others receive it
            inp.des_tpl.zero_()
            inp.kp_tpl.zero_()
        kdist.broadcast_template(inp.des_tpl, inp.kp_tpl)
    out = {}
    # 1. align_sharded with the product's HIP stages
    res = kdist.align_sharded(slabs[0], cfg, impl=kdist.HIP_STAGES)
    torch.cuda.synchronize()
    out["sharded_aligned"] = res.aligned.cpu().numpy()
    out["sharded_affines"] = res.affines
    out["sharded_skipped"] = np.asarray(res.skipped, np.int64)
    out["sharded_interpolated"] = np.asarray(res.interpolated, np.int64)
    # 2. the pipelined schedule with the two exchanges
    ov = pipeline.OverlappedSlabs(dev, cfg, counts=list(COUNTS[world]), match_beside=beside)
    r = [ov.submit(s) for s in slabs]
    rest = ov.flush()
    ov.synchronize()
    assert r[0] is None and len(rest) == 1
    for k, r in enumerate(r[1:] + rest):
        out[f"ov{k}_aligned"] = r.aligned.cpu().numpy()
        out[f"ov{k}_affines"] = r.affines
        out[f"ov{k}_skipped"] = np.asarray(r.skipped, np.int64)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    dist.destroy_process_group()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


pytestmark = pytest.mark.gpu


@pytest.mark.timeout(240)
@pytest.mark.parametrize("model,world,blind,beside", [("euclidean", 2, False, False), ("affine", 2, False, True),
                                                     ("euclidean", 3, True, False), ("affine", 3, True, True)])
def test_sharded_hip_path_equals_single_device(tmp_path, model, world, blind, beside):
    """beside: the pipelined schedule with the match on the analysis stream (c2-c4's)."""
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), str(r), str(port), str(tmp_path), model,
                               str(world), str(int(blind)), str(int(beside))],
                              env=env, cwd=REPO)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=200) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    got = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    counts = COUNTS[world]
    starts = np.concatenate(([0], np.cumsum(counts)))

    dev = torch.device("cuda", 0)
    cfg = pipeline.AlignConfig(n_kp_global=N_KP_GLOBAL, ransac_model=model)
    for s, tag in ((0, "sharded"), (0, "ov0"), (1, "ov1"), (2, "ov2")):
        ref = pipeline.align_slab(_inputs([_keypoints(r, s, model, world, blind) for r in range(world)], dev), cfg)
        if blind:  # the premise: rank 1's whole slab has no model, the gap crosses both boundaries
            assert set(range(starts[1], starts[2])) <= set(ref.skipped)
            assert set(range(starts[1], starts[2])) <= set(ref.interpolated)
        else:
            assert len(ref.skipped) < sum(counts) // 2
        aligned = ref.aligned.cpu().numpy()
        for r in range(world):
            np.testing.assert_array_equal(got[r][f"{tag}_affines"], ref.affines[starts[r]:starts[r + 1]])
        np.testing.assert_array_equal(np.concatenate([got[r][f"{tag}_aligned"] for r in range(world)]), aligned)
        if tag == "sharded":
            assert np.concatenate([got[r]["sharded_skipped"] for r in range(world)]).tolist() == ref.skipped
            assert np.concatenate([got[r]["sharded_interpolated"] for r in range(world)]).tolist() == ref.interpolated
        else:
            assert np.concatenate([got[r][f"{tag}_skipped"] for r in range(world)]).tolist() == ref.skipped


if __name__ == "__main__":
    _rank_main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]),
               bool(int(sys.argv[6])), bool(int(sys.argv[7])))
