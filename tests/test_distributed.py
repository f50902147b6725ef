"""The frame-sharded path (kcmc_amd.distributed) with world_size 2 over gloo on CPU.

The GPU kernels cannot run here, so each rank plugs CPU stand-ins built from the oracle
(test infrastructure) into the pluggable SlabStages; what is under test is the product's
sharding, the two exchange steps (survivor bitmasks, affines), the replicated native
consensus and the global post-processing: both ranks must reproduce the single-process
result exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kcmc_amd import distributed as kdist, pipeline, synthetic

F_PER_RANK, N_TPL, D, HW = 6, 80, 32, (64, 96)


def _oracle_stages(model="euclidean"):
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

    def ransac(kp_ordered, kp_tpl, pt_off, pt_idx, cfg):
        kq, kt = kp_ordered.numpy(), kp_tpl.numpy()
        out = np.full((len(pt_off) - 1,) + ((3, 3) if model == "projective" else (2, 3)), np.nan)
        for f in range(len(pt_off) - 1):
            L = pt_idx[pt_off[f]:pt_off[f + 1]]
            if len(L) >= cfg.effective_frame_skip:
                if model == "euclidean":
                    out[f] = oracle.ransac_rigid(kq[f][L], kt[L])[0]
                else:
                    out[f] = oracle.ransac_model(kq[f][L], kt[L], model)[0][: out.shape[1]]
        return torch.from_numpy(out)

    def warp(frames, affines):
        fr = frames.numpy()
        fn = oracle.warp_perspective_u16 if model == "projective" else oracle.warp_affine_u16
        return torch.from_numpy(np.stack([fn(fr[f], affines[f]) for f in range(len(fr))]))

    return kdist.SlabStages(match, ransac, warp)


def _slab(rank, n_frames, model="euclidean"):
    ks = synthetic.make_keypoints(n_frames, N_TPL, D, HW, seed=5, frame_seed=rank, model=model)
    base = synthetic.make_texture(HW, seed=1)
    frames = torch.from_numpy(np.broadcast_to(base, (n_frames,) + HW).copy())
    return pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl), torch.from_numpy(ks.kp_tpl),
                               torch.from_numpy(ks.des_q), torch.from_numpy(ks.kp_q),
                               torch.from_numpy(ks.q_off), ks.q_off)


def _worker(rank, world, port, out_dir, model):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inp = _slab(rank, F_PER_RANK + rank, model)  # uneven slabs on purpose
    if rank != 0:  # the template comes from rank 0 by broadcast
        inp.des_tpl.zero_()
        inp.kp_tpl.zero_()
    kdist.broadcast_template(inp.des_tpl, inp.kp_tpl)
    cfg = pipeline.AlignConfig(n_kp_global=20, ransac_model=model)
    res = kdist.align_sharded(inp, cfg, impl=_oracle_stages(model))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), aligned=res.aligned.numpy(), affines=res.affines,
             euclid=res.euclidean, skipped=np.array(res.skipped), interp=np.array(res.interpolated))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["euclidean", "affine", "projective"])
def test_sharded_pipeline_matches_single_process(tmp_path, model):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), model), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, f"rank{k}.npz")) for k in range(world)]
    # single-process reference over the concatenated slabs, same stages
    slabs = [_slab(k, F_PER_RANK + k, model) for k in range(world)]
    st = _oracle_stages(model)
    cfg = pipeline.AlignConfig(n_kp_global=20, ransac_model=model)
    kb, kq = zip(*[st.match(s, cfg) for s in slabs])
    keep = torch.cat(kb).numpy()
    cons = pipeline.consensus_stage(keep, N_TPL, keep.shape[0], cfg)
    params = st.ransac(torch.cat(kq), slabs[0].kp_tpl, cons.pt_off, cons.pt_idx, cfg).numpy()
    affines, skipped, interp, eu = pipeline.postprocess_affines(params, cfg)
    aligned = torch.cat([st.warp(s.frames, affines[sum(F_PER_RANK + j for j in range(k)):][: F_PER_RANK + k])
                         for k, s in enumerate(slabs)]).numpy()
    for k in range(world):
        np.testing.assert_array_equal(r[k]["affines"], affines)
        np.testing.assert_array_equal(r[k]["euclid"], eu)
        assert r[k]["skipped"].tolist() == skipped and r[k]["interp"].tolist() == interp
    np.testing.assert_array_equal(np.concatenate([r[0]["aligned"], r[1]["aligned"]]), aligned)
