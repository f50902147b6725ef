"""A/B edit (tools/ab_build.py KCMC_AB_PATCH), timing probes of the round-6 fp32 phase A of
the rigid / affine scorers (results of the probe builds are NOT correct):
  KCMC_AB_PROBE=noA2     never rescore undecided trials in fp64 (phase A2 off)
  KCMC_AB_PROBE=deadA2   phase A2's code kept, its condition never true at run time
  KCMC_AB_PROBE=nofp32   never take the fp32 path (lin32_make always false: fp64 phase A
                         with the round-6 bookkeeping)"""
import os
import sys

probe = os.environ.get("KCMC_AB_PROBE", "noA2")
for f in ("ransac.hip", "ransac_model.hip", "ransac_common.h"):
    p = os.path.join(sys.argv[1], f)
    s = open(p).read()
    if probe == "noA2":
        s = s.replace("if (!flag && und_of(v) > 0 && cnt_of(v) + und_of(v) >= mlo) {", "if (false) {")
    elif probe == "deadA2":
        s = s.replace("if (!flag && und_of(v) > 0 && cnt_of(v) + und_of(v) >= mlo) {",
                      "if (!flag && und_of(v) > 0 && cnt_of(v) + und_of(v) >= mlo + 100000) {")
    elif probe == "nofp32":
        s = s.replace("if (!(B <= 0.25 * tq) || !(tq < 1e30)) return false;", "return false;")
    open(p, "w").write(s)
