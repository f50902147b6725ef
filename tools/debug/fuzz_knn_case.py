"""Re-run one case of tests/test_gpu_fuzz.py::test_knn2_fuzz_vs_oracle and print every
template row whose (idx, dist) differs from the oracle, with the oracle's distances to the
rows involved.   python tools/debug/fuzz_knn_case.py <kind> <seed>"""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "oracle"), os.path.join(R, "tests")]
import kcmc_amd  # noqa: E402,F401
import oracle  # noqa: E402
import test_gpu_fuzz as T  # noqa: E402
from kcmc_amd import stages  # noqa: E402

kind, seed = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
rng = np.random.default_rng(2000 + 17 * seed + len(kind))
scales = []
if kind == "l2f32":
    D = int(rng.integers(1, 129))

    def gen(n):
        s = rng.choice([1e-3, 1.0, 50.0])
        scales.append(float(s))
        return rng.normal(0, s, (n, D)).astype(np.float32)
else:
    D = int(rng.integers(1, 65))
    gen = lambda n: rng.integers(0, 256, (n, D), dtype=np.uint8)  # noqa: E731
n_tpl = int(rng.integers(1, 700))
tpl = gen(n_tpl)
frames = T._frames_with_ties(rng, tpl, int(rng.integers(1, 6)), 900, gen)
print("D", D, "n_tpl", n_tpl, "rows", [len(q) for q in frames], "scales", scales)
off = np.zeros(len(frames) + 1, np.int32)
off[1:] = np.cumsum([len(q) for q in frames])
des_q = np.concatenate(frames)
idx, dist = stages.knn2_l2u8(T._t(tpl, dev), T._t(des_q, dev), T._t(off, dev), int(np.diff(off).max()))
idx, dist = idx.cpu().numpy(), dist.cpu().numpy()
ora = oracle.knn2_l2f32 if kind == "l2f32" else oracle.knn2_l2u8
for f, q in enumerate(frames):
    ri, rd = ora(tpl, q)
    bad = np.flatnonzero((idx[f] != ri).any(1) | (dist[f].view(np.int32) != rd.view(np.int32)).any(1))
    print(f"frame {f}: {len(q)} rows, {len(bad)} template rows differ")
    for i in bad[:10]:
        ex = [float(np.sqrt(np.float32(np.sum((tpl[i].astype(np.float64) - q[j].astype(np.float64)) ** 2))))
              for j in range(len(q))]
        print(f"  tpl {i}: got {idx[f, i].tolist()} {dist[f, i].tolist()}  oracle {ri[i].tolist()} {rd[i].tolist()}"
              f"  all dists {np.round(ex, 6).tolist()[:8]}")
