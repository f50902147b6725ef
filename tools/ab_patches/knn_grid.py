"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the u8 matcher's persistent grid at a fraction
of full residency, KCMC_AB_KNN_DIV (default 2) -- leaves wave slots and LDS to the warp
tiles that run beside the match in the pipelined schedule."""
import os
import sys

p = os.path.join(sys.argv[1], "match.hip")
s = open(p).read()
a = "dim3(knn_grid(n_tg, n_frames, per_cu))"
assert a in s
div = int(os.environ.get("KCMC_AB_KNN_DIV", "2"))
s = s.replace(a, f"dim3(knn_grid(n_tg, n_frames, std::max(1, per_cu / {div})))")
open(p, "w").write(s)
