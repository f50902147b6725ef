// CU-mask layout lab (not part of the library): which physical CU does each bit of a
// hipExtStreamCreateWithCUMask mask select?  Only masks with exactly ONE bit cleared are
// launched, so every XCD and shader engine keeps CUs (a mask that leaves an XCD without
// CUs is the suspected cause of the 180 s stall recorded in DESIGN.md; it is not run).
//
// Build here:  hipcc --offload-arch=gfx950 -O3 tools/cu_mask_lab.hip -o ab/cu_mask_lab
// Run on the box (bounded):  timeout -k 10 120 ./ab/cu_mask_lab > gpurun_out/cu_mask.txt
//
// Each workgroup records its HW_ID (CU_ID [11:8], SH_ID [12], SE_ID [15:13]) and XCC_ID
// (s_getreg: hardware-register reads into SGPRs, stored with a vector store) and sleeps a
// few microseconds so that a launch of 4096 workgroups spreads over every enabled CU.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void where_kernel(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  for (int k = 0; k < 4; ++k) __builtin_amdgcn_s_sleep(127);
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e));                         \
      return 1;                                                             \
    }                                                                       \
  } while (0)

using CU = std::tuple<int, int, int, int>;  // xcc, se, sh, cu

static int run(hipStream_t s, uint32_t* d, std::vector<uint32_t>& h, int nwg, std::set<CU>& seen) {
  hipLaunchKernelGGL(where_kernel, dim3(nwg), dim3(64), 0, s, d);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  seen.clear();
  for (int b = 0; b < nwg; ++b) {
    const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    seen.insert(CU((int)xcc, (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 15)));
  }
  return 0;
}

int main() {
  const int nwg = 4096;
  uint32_t* d;
  CK(hipMalloc(&d, nwg * 8));
  std::vector<uint32_t> h(2 * nwg);
  std::set<CU> all, seen;
  if (run(0, d, h, nwg, all)) return 1;
  printf("default queue: %zu distinct CUs\n", all.size());
  fflush(stdout);
  for (int bit = 0; bit < 256; ++bit) {
    uint32_t mask[8];
    for (auto& m : mask) m = 0xffffffffu;
    mask[bit >> 5] &= ~(1u << (bit & 31));
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, 8, mask));
    if (run(s, d, h, nwg, seen)) return 1;
    CK(hipStreamDestroy(s));
    std::vector<CU> missing;
    for (const CU& c : all)
      if (!seen.count(c)) missing.push_back(c);
    printf("bit %3d: %zu CUs;", bit, seen.size());
    for (const CU& c : missing)
      printf(" missing xcc %d se %d sh %d cu %d", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
    printf("\n");
    fflush(stdout);
  }
  CK(hipFree(d));
  return 0;
}
