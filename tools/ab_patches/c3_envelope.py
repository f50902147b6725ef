"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the c3 analysis kernels sized to the slot a CU
full of warp tiles leaves (7 workgroups x 4 waves of the one-channel warp: one wave slot per
SIMD, 120 VGPRs, 20 KB of LDS).  KCMC_AB_ENVELOPE = "knn", "ransac" or "knn,ransac":
  knn:    the u8 matcher at 4 waves per workgroup for every n_tpl, 96-row staged chunks
          (2 x 96 x 80 B + keys = 16 KB LDS), <= 120 VGPRs, one workgroup per CU on its
          persistent grid (so the warp keeps the other slots);
  ransac: the affine RANSAC scoring at 5 waves per SIMD (launch bounds: <= 102 VGPRs;
          amdgpu_num_vgpr(120) is not honoured here, the scoring stays at 122)."""
import os
import sys

what = os.environ.get("KCMC_AB_ENVELOPE", "knn,ransac").split(",")
d = sys.argv[1]
if "knn" in what:
    p = os.path.join(d, "match.hip")
    s = open(p).read()
    for a, b in (("constexpr int kQChunk = 256;", "constexpr int kQChunk = 96;"),
                 ("__global__ __launch_bounds__(KnnShape<WAVES>::kThreads) void knn2_l2u8_kernel(",
                  "__global__ __launch_bounds__(KnnShape<WAVES>::kThreads) __attribute__((amdgpu_num_vgpr(120))) "
                  "void knn2_l2u8_kernel("),
                 ("dim3(knn_grid(n_tg, n_frames, per_cu))", "dim3(knn_grid(n_tg, n_frames, 1))"),
                 ("const bool wide = n_tpl > 256;", "const bool wide = false;")):
        assert a in s, a
        s = s.replace(a, b)
    open(p, "w").write(s)
if "ransac" in what:
    p = os.path.join(d, "ransac_model.hip")
    s = open(p).read()
    a = "__global__ __launch_bounds__(kThreads, MODEL == KCMC_MODEL_AFFINE ? 1 : 2) void\nransac_model_score_kernel("
    assert a in s
    s = s.replace(a, "__global__ __launch_bounds__(kThreads, MODEL == KCMC_MODEL_AFFINE ? 5 : 2) void\n"
                     "ransac_model_score_kernel(")
    open(p, "w").write(s)
