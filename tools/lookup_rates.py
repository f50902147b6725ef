"""Time the device consensus lookup alone (kcmc_consensus_lookup: count + scan + order
kernels) on c2 / c3-shaped survivor bitmasks; same-box A/B with KCMC_LIB_PATH=ab/<name>.so.

    python tools/lookup_rates.py [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcmc_amd import stages  # noqa: E402


def case(F, n_tpl, density, nkg, reps, dev):
    rng = np.random.default_rng(F + n_tpl)
    words = (n_tpl + 31) // 32
    on = np.zeros((F, words * 32), bool)
    on[:, :n_tpl] = rng.random((F, n_tpl)) < density
    kb = np.ascontiguousarray(np.packbits(on, axis=1, bitorder="little")).view(np.uint32)
    v = stages.consensus_vote_host(kb, n_tpl)
    choice = stages.consensus_merge(v, n_tpl, nkg, 1)
    kbd = torch.from_numpy(kb.view(np.int32)).to(dev)
    pack = torch.from_numpy(choice.pack).to(dev)
    for _ in range(3):
        po, pi = stages.consensus_lookup(kbd, n_tpl, pack, choice.nc)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        po, pi = stages.consensus_lookup(kbd, n_tpl, pack, choice.nc)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    h = int(np.bitwise_xor.reduce(pi.cpu().numpy()[: int(po[-1])].astype(np.int64) * 2654435761 % (1 << 31)))
    print(f"F {F} n_tpl {n_tpl} density {density} nc {choice.nc}: median {np.median(ts) * 1e3:.1f} us "
          f"min {min(ts) * 1e3:.1f} us (points {int(po[-1])}, hash {h})", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    case(2500, 500, 0.6, 50, reps, dev)    # c3
    case(2000, 500, 0.6, 100, reps, dev)   # c2
    case(625, 4096, 0.3, 500, reps, dev)   # c4
    case(500, 4096, 0.3, 200, reps, dev)   # c5


if __name__ == "__main__":
    main()
