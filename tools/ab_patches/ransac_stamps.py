"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): phase timestamps of the rigid scorer, a
timing instrument (never the product library; tools/debug/ransac_stamps.py reads them).

Thread 0 of every frame's workgroup records s_memtime right after the barriers that end
each phase, plus two counters kept in LDS (trials re-counted by phase A2, phase-B
candidates) and whether the frame fell back to exact scoring:
  0 entry   1 staged (points + magnitudes in LDS)   2 phase A (fp32 counts + brackets)
  3 phase A2 (fp64 re-counts)   4 best count known   5 phase B + argmax   6 selection
  7 end (inlier mask + refit)   8 A2 trials   9 phase-B candidates   10 exact path
Stamps go to a __device__ array through ordinary vector stores; kcmc_debug_ransac_stamps
copies them out (hipMemcpyFromSymbol)."""
import os
import sys

p = os.path.join(sys.argv[1], "ransac.hip")
s = open(p).read()


def sub(a, b, count=1):
    global s
    assert s.count(a) == count, (a, s.count(a))
    s = s.replace(a, b)


sub("using namespace ransac_common;\n",
    "using namespace ransac_common;\n\n"
    "constexpr int kStampFrames = 8192, kStamps = 12;\n"
    "__device__ unsigned long long g_stamps[kStampFrames * kStamps];\n"
    "#define STAMP(i) do { if (tid == 0 && f < kStampFrames) g_stamps[(size_t)f * kStamps + (i)] = "
    "__builtin_amdgcn_s_memtime(); } while (0)\n"
    "#define STAMP_V(i, v) do { if (tid == 0 && f < kStampFrames) g_stamps[(size_t)f * kStamps + (i)] = "
    "(unsigned long long)(v); } while (0)\n")
# entry (before the early returns of skipped frames: those record only the entry)
sub("  const int tid = threadIdx.x;\n  const int lane = tid & 63, wave = tid >> 6;\n  const int p0 = pt_off[f];\n",
    "  const int tid = threadIdx.x;\n  const int lane = tid & 63, wave = tid >> 6;\n  STAMP(0);\n"
    "  __shared__ int s_na2, s_nb;\n  if (tid == 0) { s_na2 = 0; s_nb = 0; }\n  const int p0 = pt_off[f];\n")
sub("  for (int k = tid; k < N; k += kThreads) pk32[k] = centred32(sx[k], sy[k], dxs[k], dys[k], mg);\n  __syncthreads();\n",
    "  for (int k = tid; k < N; k += kThreads) pk32[k] = centred32(sx[k], sy[k], dxs[k], dys[k], mg);\n  __syncthreads();\n"
    "  STAMP(1);\n")
sub("    __syncthreads();  // s_cnt is reused\n", "    __syncthreads();  // s_cnt is reused\n    STAMP(2);\n")
sub("        const int tc = t0 + __builtin_ctzll(need);\n",
    "        const int tc = t0 + __builtin_ctzll(need);\n        if (lane == 0) atomicAdd(&s_na2, 1);\n")
sub("    __syncthreads();  // the A2 results of the other waves' lanes\n",
    "    __syncthreads();  // the A2 results of the other waves' lanes\n    STAMP(3);\n")
sub("  const bool exact = flag != 0 || mcount <= 0;\n",
    "  const bool exact = flag != 0 || mcount <= 0;\n  STAMP(4);\n  STAMP_V(10, exact ? 1 : 0);\n")
sub("        const int tc = t0 + __builtin_ctzll(cand);\n",
    "        const int tc = t0 + __builtin_ctzll(cand);\n        if (lane == 0) atomicAdd(&s_nb, 1);\n")
sub("  if (any_zero) atomicOr(&s_any_zero, 1);\n  __syncthreads();\n",
    "  if (any_zero) atomicOr(&s_any_zero, 1);\n  __syncthreads();\n  STAMP(5);\n")
sub("  __syncthreads();\n  const int best_t = s_final_t;\n",
    "  __syncthreads();\n  STAMP(6);\n  const int best_t = s_final_t;\n")
sub("    out_nin[f] = (int32_t)n_in;\n    out_best[f] = best_t;\n  }\n",
    "    out_nin[f] = (int32_t)n_in;\n    out_best[f] = best_t;\n  }\n  STAMP(7);\n  STAMP_V(8, s_na2);\n"
    "  STAMP_V(9, s_nb);\n")
s += ("\nextern \"C\" int kcmc_debug_ransac_stamps(void* dst, int n_frames) {\n"
      "  const size_t n = (size_t)(n_frames < kcmc::kStampFrames ? n_frames : kcmc::kStampFrames) * kcmc::kStamps;\n"
      "  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(kcmc::g_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess"
      " ? 0 : -1;\n}\n")
open(p, "w").write(s)
