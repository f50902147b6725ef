"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the rigid and affine scorers at 3 waves per
SIMD (up to 168 VGPRs, no spills) instead of 4 (128 VGPRs)."""
import os
import sys

for f, a, b in (("ransac.hip", "__launch_bounds__(kThreads, 4) void ransac_rigid_kernel(",
                 "__launch_bounds__(kThreads, 3) void ransac_rigid_kernel("),
                ("ransac_model.hip", "MODEL == KCMC_MODEL_AFFINE ? 4 : 2", "MODEL == KCMC_MODEL_AFFINE ? 3 : 2")):
    p = os.path.join(sys.argv[1], f)
    s = open(p).read()
    assert a in s, a
    open(p, "w").write(s.replace(a, b))
