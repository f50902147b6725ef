"""The frame-sharded path (kcmc_amd.distributed) with world_size 2 and 3 over gloo on CPU.

The GPU kernels cannot run here, so each rank plugs CPU stand-ins into the pluggable
SlabStages: the oracle's matcher / RANSAC / warp (test infrastructure) and the product's
native host consensus parts (kcmc_consensus_vote_host / _lookup_host, the same definitions
as the device kernels).  What is under test is the product's sharding: the vote exchange
(O(n_tpl) per rank), the host merge every rank makes, the per-rank lookup, the slab-boundary
exchange and the per-rank NaN-gap filling -- the ranks' results, concatenated, must equal
the single-process result exactly, also when a whole rank's slab has no model (gaps that
cross rank boundaries, leading / trailing gaps owned by other ranks)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kcmc_amd import distributed as kdist, pipeline, stages, synthetic

F_PER_RANK, N_TPL, D, HW = 6, 80, 32, (64, 96)


def _boundary_np(params: torch.Tensor) -> torch.Tensor:
    p = params.numpy().reshape(len(params), -1)
    E = p.shape[1]
    ok = np.flatnonzero(~np.isnan(p).any(axis=1))
    out = np.full(2 + 2 * E, np.nan)
    out[:2] = (ok[0], ok[-1]) if ok.size else (-1, -1)
    if ok.size:
        out[2:2 + E], out[2 + E:] = p[ok[0]], p[ok[-1]]
    return torch.from_numpy(out)


def _oracle_stages(model="euclidean", no_model=False):
    """no_model: this rank's RANSAC fails on every frame (NaN parameters)."""
    import oracle

    def match(inp, cfg):
        qo = inp.q_off_host
        des_t, kp_t = inp.des_tpl.numpy(), inp.kp_tpl.numpy()
        bits = np.zeros((len(qo) - 1, (N_TPL + 31) // 32), np.uint32)
        kq_all = np.zeros((len(qo) - 1, N_TPL, 2))
        for f in range(len(qo) - 1):
            idx, dist_ = oracle.knn2_l2u8(des_t, inp.des_q.numpy()[qo[f]:qo[f + 1]])
            s, kq, _ = oracle.filter_matches(idx, dist_, kp_t, inp.kp_q.numpy()[qo[f]:qo[f + 1]])
            for i in s:
                bits[f, i >> 5] |= np.uint32(1 << (i & 31))
            kq_all[f] = kq
        return torch.from_numpy(bits.view(np.int32)), torch.from_numpy(kq_all)

    def vote(keep_bits, n_tpl, frame_base):
        return torch.from_numpy(stages.consensus_vote_host(keep_bits.numpy(), n_tpl, frame_base))

    def lookup(keep_bits, n_tpl, choice):
        pt_off, pt_idx = stages.consensus_lookup_host(keep_bits.numpy(), n_tpl, choice.cons_iter)
        return stages.Consensus(choice.order, choice.votes, pt_off, pt_idx)

    def ransac(kp_ordered, kp_tpl, cons, cfg):
        kq, kt = kp_ordered.numpy(), kp_tpl.numpy()
        out = np.full((len(cons.pt_off) - 1,) + ((3, 3) if model == "projective" else (2, 3)), np.nan)
        for f in range(len(cons.pt_off) - 1):
            L = cons.pt_idx[cons.pt_off[f]:cons.pt_off[f + 1]]
            if len(L) >= cfg.effective_frame_skip and not no_model:
                if model == "euclidean":
                    out[f] = oracle.ransac_rigid(kq[f][L], kt[L])[0]
                else:
                    out[f] = oracle.ransac_model(kq[f][L], kt[L], model)[0][: out.shape[1]]
        return torch.from_numpy(out)

    def warp(frames, affines):
        fr = frames.numpy()
        fn = oracle.warp_perspective_u16 if model == "projective" else oracle.warp_affine_u16
        return torch.from_numpy(np.stack([fn(fr[f], affines[f]) for f in range(len(fr))]))

    def warp_params(frames, params):  # the HIP warp's contract: a frame without a model -> zeros
        p = params.numpy()
        out = warp(frames, np.nan_to_num(p)).numpy()
        out[np.isnan(p).reshape(len(p), -1).any(axis=1)] = 0
        return torch.from_numpy(out)

    return kdist.SlabStages(match, vote, lookup, ransac, _boundary_np, warp, warp_params)


def _slab(rank, n_frames, model="euclidean"):
    ks = synthetic.make_keypoints(n_frames, N_TPL, D, HW, seed=5, frame_seed=rank, model=model)
    base = synthetic.make_texture(HW, seed=1)
    frames = torch.from_numpy(np.broadcast_to(base, (n_frames,) + HW).copy())
    return pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl), torch.from_numpy(ks.kp_tpl),
                               torch.from_numpy(ks.des_q), torch.from_numpy(ks.kp_q),
                               torch.from_numpy(ks.q_off), ks.q_off)


def _worker(rank, world, port, out_dir, model, nan_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp = _slab(rank, F_PER_RANK + rank, model)  # uneven slabs on purpose
    if rank != 0:  # the template comes from rank 0 by broadcast
        inp.des_tpl.zero_()
        inp.kp_tpl.zero_()
    kdist.broadcast_template(inp.des_tpl, inp.kp_tpl)
    cfg = pipeline.AlignConfig(n_kp_global=20, ransac_model=model)
    res = kdist.align_sharded(inp, cfg, impl=_oracle_stages(model, no_model=rank == nan_rank))
    counts = [F_PER_RANK + r for r in range(world)]
    g_aff, g_eu, g_sk, g_it = kdist.gather_results(res, counts)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), aligned=res.aligned.numpy(), affines=res.affines,
             euclid=res.euclidean, skipped=np.array(res.skipped, np.int64),
             interp=np.array(res.interpolated, np.int64), f0=res.extras["f0"], order=res.consensus.order,
             g_aff=g_aff, g_eu=g_eu, g_sk=np.array(g_sk, np.int64), g_it=np.array(g_it, np.int64))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,world,nan_rank", [("euclidean", 2, None), ("affine", 2, None), ("projective", 2, None),
                                                  ("euclidean", 3, 1), ("euclidean", 3, 0), ("euclidean", 3, 2),
                                                  ("affine", 3, 1)])
def test_sharded_pipeline_matches_single_process(tmp_path, model, world, nan_rank):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), model, nan_rank), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, f"rank{k}.npz")) for k in range(world)]
    # single-process reference over the concatenated slabs, same stages, the host consensus
    counts = [F_PER_RANK + k for k in range(world)]
    slabs = [_slab(k, counts[k], model) for k in range(world)]
    st = _oracle_stages(model)
    cfg = pipeline.AlignConfig(n_kp_global=20, ransac_model=model)
    kb, kq = zip(*[st.match(s, cfg) for s in slabs])
    keep = torch.cat(kb).numpy()
    cons = pipeline.consensus_stage(keep, N_TPL, keep.shape[0], cfg)
    params = st.ransac(torch.cat(kq), slabs[0].kp_tpl, cons, cfg).numpy()
    if nan_rank is not None:
        params[sum(counts[:nan_rank]):sum(counts[:nan_rank + 1])] = np.nan
    affines, skipped, interp, eu = pipeline.postprocess_affines(params, cfg)
    starts = np.concatenate(([0], np.cumsum(counts)))
    aligned = torch.cat([st.warp(s.frames, affines[starts[k]:starts[k + 1]]) for k, s in enumerate(slabs)]).numpy()
    if nan_rank == 1:
        assert any(starts[1] <= i < starts[2] for i in interp)  # the gap crosses both rank boundaries
    for k in range(world):
        assert int(r[k]["f0"]) == starts[k]
        np.testing.assert_array_equal(r[k]["order"], cons.order)
        np.testing.assert_array_equal(r[k]["affines"], affines[starts[k]:starts[k + 1]])
        np.testing.assert_array_equal(r[k]["euclid"], eu[starts[k]:starts[k + 1]])
        assert r[k]["skipped"].tolist() == [i for i in skipped if starts[k] <= i < starts[k + 1]]
        assert r[k]["interp"].tolist() == [i for i in interp if starts[k] <= i < starts[k + 1]]
        np.testing.assert_array_equal(r[k]["g_aff"], affines)
        np.testing.assert_array_equal(r[k]["g_eu"], eu)
        assert r[k]["g_sk"].tolist() == skipped and r[k]["g_it"].tolist() == interp
    np.testing.assert_array_equal(np.concatenate([r[k]["aligned"] for k in range(world)]), aligned)
