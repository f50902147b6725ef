"""Stress the 4K RGB warp (test_config4's frames and maps): N warps into fresh allocations,
each checked against the oracle; on a mismatch the positions, a re-read of the device buffer
and the cache-line offsets are logged.  python tools/debug/c4_warp_stress.py <tag> [reps]"""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "oracle"))
import oracle  # noqa: E402
from kcmc_amd import pipeline  # noqa: E402
from test_gpu_configs import _texture  # noqa: E402

tag = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
out_dir = os.path.join(R, "gpurun_out", "dbg_c4_stress")
os.makedirs(out_dir, exist_ok=True)
dev = torch.device("cuda:0")
F, H, W, C = 3, 2160, 3840, 3
A = np.array([[[1.0053911383577487, 0.0057811368368455435, 1.2748370385747876],
               [-0.014055324654216174, 0.9906779338198224, -0.4287047332629754]],
              [[1.0078828926080385, 0.006215137383056257, -3.653160507510165],
               [-0.006516371002192053, 0.9984373506161567, 1.0913358526368029]],
              [[1.0045123939733775, 0.0051991689442833, -0.7138911485271819],
               [-0.0003428726917676483, 1.0085363575053359, -4.207238076060094]]])
base = _texture(H, W, C, 44)
refs = [oracle.warp_affine_u16(base, A[f]) for f in range(F)]
frames = torch.from_numpy(np.broadcast_to(base, (F,) + base.shape).copy()).to(dev)
maps = torch.from_numpy(A).to(dev)
lines = []
n_bad = 0
for rep in range(reps):
    o_dev = pipeline.warp_frames(frames, maps)
    o = o_dev.cpu().numpy()
    for f in range(F):
        bad = np.argwhere(o[f] != refs[f])
        if len(bad):
            n_bad += 1
            again = o_dev[f].cpu().numpy()[tuple(bad.T)]
            exp = refs[f][tuple(bad.T)]
            byte = ((bad[:, 0] * W + bad[:, 1]) * C + bad[:, 2]) * 2
            lines.append(f"rep {rep} frame {f}: {len(bad)} mismatches; re-read equal to the oracle "
                         f"{int((again == exp).sum())}; 128-B lines {sorted(set((byte // 128).tolist()))[:8]}; "
                         f"first (y,x,c) {bad[:4].tolist()} got {o[f][tuple(bad[:8].T)].tolist()} "
                         f"exp {exp[:8].tolist()}")
            print(lines[-1], flush=True)
    del o_dev
print(f"{tag}: {reps} reps x {F} frames, {n_bad} bad frame outputs", flush=True)
open(os.path.join(out_dir, f"{tag}.txt"), "w").write("\n".join(lines + [f"{tag}: {reps} reps, {n_bad} bad"]) + "\n")
