"""Diagnose a c4 (4K RGB) warp mismatch: the slab of tests/test_gpu_configs.py
test_config4_4k_rgb_affine_slab, then the warp alone on the same maps, repeated, against the
oracle.  Writes gpurun_out/dbg_c4/summary.txt."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "oracle"))
import oracle  # noqa: E402
from kcmc_amd import pipeline, synthetic  # noqa: E402
from test_gpu_configs import _texture  # noqa: E402

out_dir = os.path.join(R, "gpurun_out", "dbg_c4")
os.makedirs(out_dir, exist_ok=True)
lines = []


def log(*a):
    s = " ".join(str(x) for x in a)
    print(s, flush=True)
    lines.append(s)


dev = torch.device("cuda:0")
F, H, W, C = 3, 2160, 3840, 3
ks = synthetic.make_keypoints(F, 4096, 61, (H, W), seed=43, model="affine", descriptor="u8")
base = _texture(H, W, C, 44)
frames = torch.from_numpy(np.broadcast_to(base, (F,) + base.shape).copy()).to(dev)
inp = pipeline.SlabInputs(frames, torch.from_numpy(ks.des_tpl).to(dev), torch.from_numpy(ks.kp_tpl).to(dev),
                          torch.from_numpy(ks.des_q).to(dev), torch.from_numpy(ks.kp_q).to(dev),
                          torch.from_numpy(ks.q_off).to(dev), ks.q_off)
cfg = pipeline.AlignConfig(n_kp_global=500, ransac_model="affine")
res = pipeline.align_slab(inp, cfg, keep_intermediates=True)
torch.cuda.synchronize()
params = res.ransac.params.cpu().numpy()
log("params (device RANSAC):", params.tolist())
log("affines (host):", np.asarray(res.affines).tolist())
log("skipped", res.skipped, "interpolated", res.interpolated)
out = res.aligned.cpu().numpy()
refs = {}
for f in range(F):
    ref = oracle.warp_affine_u16(base, np.asarray(res.affines[f]))
    refs[f] = ref
    bad = np.argwhere(out[f] != ref)
    log(f"slab frame {f}: mismatches {len(bad)}", bad[:10].tolist() if len(bad) else "")
    if len(bad):
        ys, xs = bad[:, 0], bad[:, 1]
        log(f"  rows {ys.min()}..{ys.max()} cols {xs.min()}..{xs.max()}; tiles (x/128, y/24):",
            sorted(set(zip((xs // 128).tolist(), (ys // 24).tolist())))[:20])
        d = out[f].astype(np.int64) - ref.astype(np.int64)
        log("  max |diff|", int(np.abs(d).max()))
        np.save(os.path.join(out_dir, f"bad_{f}.npy"), bad[:2000])
# the warp alone on the same maps, repeated, into fresh torch allocations (out=None, the
# mode that failed); on a mismatch the same device buffer is read back a second time
# (a stale first read vs wrong values in memory) and the positions are saved
maps = torch.from_numpy(np.ascontiguousarray(np.asarray(res.affines, dtype=np.float64))).to(dev)
keep = []
for rep in range(12):
    o_dev = pipeline.warp_frames(frames, maps)
    o = o_dev.cpu().numpy()
    for f in range(F):
        bad = np.argwhere(o[f] != refs[f])
        if len(bad):
            got = o[f][tuple(bad.T)]
            exp = refs[f][tuple(bad.T)]
            again = o_dev[f].cpu().numpy()[tuple(bad.T)]
            torch.cuda.synchronize()
            again2 = o_dev[f].cpu().numpy()[tuple(bad.T)]
            log(f"rep {rep} frame {f}: mismatches {len(bad)}; second read equal to the oracle: "
                f"{int((again == exp).sum())}/{len(bad)}, third: {int((again2 == exp).sum())}")
            log("   positions (y, x, c):", bad[:64].tolist())
            log("   got:", got[:64].tolist())
            log("   exp:", exp[:64].tolist())
            np.save(os.path.join(out_dir, f"rep{rep}_f{f}.npy"), np.concatenate([bad, got[:, None], exp[:, None]], 1))
        else:
            log(f"rep {rep} frame {f}: ok")
    keep.append(o_dev)  # hold every output: each rep gets fresh memory
open(os.path.join(out_dir, "summary.txt"), "w").write("\n".join(lines) + "\n")
