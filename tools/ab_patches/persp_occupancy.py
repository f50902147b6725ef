"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the perspective warp's tile kernel launched with
KCMC_AB_PERSP_PAD bytes of extra (unused) dynamic LDS per workgroup, so fewer of its
workgroups fit a CU and wave slots stay free for the kernels beside it (RANSAC, the float
matcher's tile images)."""
import os
import sys

p = os.path.join(sys.argv[1], "warp.hip")
s = open(p).read()
a = "dim3(ntx, nty, n_frames), dim3(kThreads), 0, s, src, dst,\n                     plan, minv"
assert a in s
pad = int(os.environ.get("KCMC_AB_PERSP_PAD", "3072"))
s = s.replace(a, a.replace("dim3(kThreads), 0, s", f"dim3(kThreads), {pad}, s"))
open(p, "w").write(s)
