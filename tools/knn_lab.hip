// Ablation lab for the K1 matchers (not part of the library).  Times launch_knn of a
// (possibly edited) copy of match.hip on synthetic uint8 descriptors, or with -DKNN_F32
// launch_knn_f32 of match_f32.hip on SIFT-style float descriptors (unit-normalised
// Gaussian template rows; frame rows = 80 % noisy template rows (sigma 0.05), 20 % fresh
// unit vectors, like kcmc_amd/synthetic.py).  Build here:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude tools/knn_lab.hip -o ab/knn_lab
//   (-DMATCH_SRC='"path"' builds it against an edited copy: tools/knn_lab.sh makes the ablations)
// Run on the GPU box:  ab/knn_lab [n_tpl D frames n_q reps]   (default: config 4, 4096 61 625 4506 10;
//                      f32: config 5, 4096 128 500 4500 5)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"
namespace kcmc {
void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }
int fail(int c, const std::string& m) { set_error(m); return c; }
int hip_check(hipError_t e, const char* w) { if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e)); return KCMC_EHIP; } return 0; }
int launch_check(const char* w) { return hip_check(hipGetLastError(), w); }
// one cached workspace (the library's is a per-context pool): no allocation in the timed region
static void* g_ws = nullptr;
static size_t g_ws_size = 0;
int workspace_alloc(kcmc_ctx*, void** p, size_t n, hipStream_t) {
  if (n > g_ws_size) {
    if (g_ws) (void)hipFree(g_ws);
    g_ws = nullptr;
    g_ws_size = 0;
    if (int e = hip_check(hipMalloc(&g_ws, n), "ws")) return e;
    g_ws_size = n;
  }
  *p = g_ws;
  return 0;
}
int workspace_free(kcmc_ctx*, void*, hipStream_t, size_t) { return 0; }
#ifdef KNN_F32  // match_f32.hip's kcmc_match_frames_f32 calls match.hip's filter launcher
int device_cus() {
  int d = 0, n = 256;
  (void)hipGetDevice(&d);
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
  return n;
}
int launch_match_filter(const int32_t*, const float*, const double*, const double*, const int32_t*, int, int, double,
                        double, double, double*, uint32_t*, int32_t*, hipStream_t) {
  return KCMC_EUNSUPPORTED;
}
#endif
}  // namespace kcmc
#ifdef KNN_F32
#ifndef MATCH_SRC
#define MATCH_SRC "../keypoint-consensus-motion-correction_amd/csrc/match_f32.hip"
#endif
typedef float Desc;
#else
#ifndef MATCH_SRC
#define MATCH_SRC "../keypoint-consensus-motion-correction_amd/csrc/match.hip"
#endif
typedef uint8_t Desc;
#endif
#include MATCH_SRC
#include <cmath>

static int launch(const Desc* t, int n_tpl, int D, const Desc* q, const int32_t* off, int F, int nq, int32_t* idx,
                  float* dist) {
#ifdef KNN_F32
  return kcmc::launch_knn_f32(nullptr, t, n_tpl, D, q, off, F, nq, nullptr, idx, dist, 0);
#else
  return kcmc::launch_knn(t, n_tpl, D, q, off, F, nq, idx, dist, 0);
#endif
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e = (x);                                            \
    if (e != hipSuccess) {                                         \
      printf("%s: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
#ifdef KNN_F32
  const int n_tpl = argc > 1 ? atoi(argv[1]) : 4096;
  const int D = argc > 2 ? atoi(argv[2]) : 128;
  const int F = argc > 3 ? atoi(argv[3]) : 500;
  const int nq = argc > 4 ? atoi(argv[4]) : 4500;
  const int reps = argc > 5 ? atoi(argv[5]) : 5;
  const int maxD = 128;
#else
  const int n_tpl = argc > 1 ? atoi(argv[1]) : 4096;
  const int D = argc > 2 ? atoi(argv[2]) : 61;
  const int F = argc > 3 ? atoi(argv[3]) : 625;
  const int nq = argc > 4 ? atoi(argv[4]) : 4506;
  const int reps = argc > 5 ? atoi(argv[5]) : 10;
  const int maxD = 64;
#endif
  if (n_tpl < 1 || n_tpl > 8192 || D < 1 || D > maxD || F < 1 || nq < 2 || (size_t)F * nq * D > (1ull << 31)) {
    printf("bad shape\n");
    return 1;
  }
  std::vector<Desc> tpl((size_t)n_tpl * D), q((size_t)F * nq * D);
  uint32_t s = 12345u;
  auto u01 = [&]() { return ((s = s * 1664525u + 1013904223u) >> 8) * (1.0 / 16777216.0) + 1e-9; };
#ifdef KNN_F32
  auto gauss = [&]() { return sqrt(-2.0 * log(u01())) * cos(6.283185307179586 * u01()); };
  auto unit_row = [&](float* r) {
    double n2 = 0;
    for (int k = 0; k < D; ++k) n2 += (r[k] = (float)gauss()) * (double)r[k];
    for (int k = 0; k < D; ++k) r[k] = (float)(r[k] / sqrt(n2));
  };
  for (int i = 0; i < n_tpl; ++i) unit_row(&tpl[(size_t)i * D]);
  for (size_t j = 0; j < (size_t)F * nq; ++j) {
    float* r = &q[j * D];
    if (u01() < 0.8) {
      const size_t i = (size_t)(u01() * n_tpl) % n_tpl;
      for (int k = 0; k < D; ++k) r[k] = tpl[i * D + k] + (float)(0.05 * gauss());
    } else {
      unit_row(r);
    }
  }
#else
  for (auto& v : tpl) v = (uint8_t)((s = s * 1664525u + 1013904223u) >> 24);
  for (auto& v : q) v = (uint8_t)((s = s * 1664525u + 1013904223u) >> 24);
#endif
  std::vector<int32_t> off(F + 1);
  for (int f = 0; f <= F; ++f) off[f] = f * nq;
  Desc *d_tpl, *d_q;
  int32_t *d_off, *d_idx;
  float* d_dist;
  CK(hipMalloc(&d_tpl, tpl.size() * sizeof(Desc)));
  CK(hipMalloc(&d_q, q.size() * sizeof(Desc)));
  CK(hipMalloc(&d_off, off.size() * 4));
  CK(hipMalloc(&d_idx, (size_t)F * n_tpl * 2 * 4));
  CK(hipMalloc(&d_dist, (size_t)F * n_tpl * 2 * 4));
  CK(hipMemcpy(d_tpl, tpl.data(), tpl.size() * sizeof(Desc), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_q, q.data(), q.size() * sizeof(Desc), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  if (launch(d_tpl, n_tpl, D, d_q, d_off, F, nq, d_idx, d_dist)) return 1;
  CK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0.f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    if (launch(d_tpl, n_tpl, D, d_q, d_off, F, nq, d_idx, d_dist)) return 1;
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
    sum += ms;
  }
  std::vector<int32_t> idx((size_t)F * n_tpl * 2);
  CK(hipMemcpy(idx.data(), d_idx, idx.size() * 4, hipMemcpyDeviceToHost));
  unsigned long long ck = 0;
  for (size_t i = 0; i < idx.size(); ++i) ck = ck * 1000003ull + (uint32_t)idx[i];
  const double ops = 2.0 * n_tpl * (double)nq * D * F;
  long n_fb = -1;  // the float matcher's fallback rows (its per-frame counters head the workspace)
#ifdef KNN_F32
  std::vector<int32_t> cnt(F);
  CK(hipMemcpy(cnt.data(), g_ws, (size_t)F * 4, hipMemcpyDeviceToHost));
  n_fb = 0;
  for (int32_t c : cnt) n_fb += c;
#endif
#ifdef KCMC_STAMP
  {
    unsigned long long st[8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st)));
    const double w = (double)st[4], tl = (double)st[5];
    printf("stamps (s_memtime ticks, all launches): per wave and %s: %s %.1f, barrier %.1f, total %.1f; "
           "waves %.0f %ss/wave %.2f\n",
#ifdef KNN_F32
           "tile", "vmcnt wait", st[0] / tl, st[1] / tl, st[2] / tl, w, "tile", tl / w);
#else
           "chunk", "staging (land_row)", st[0] / tl, st[1] / tl, st[2] / tl, w, "chunk", tl / w);
#endif
  }
#endif
  printf("n_tpl %d D %d F %d nq %d: best %.4f ms mean %.4f ms (%.1f TOPs algorithmic) idx-hash %016llx fallback %ld\n",
         n_tpl, D, F, nq, best, sum / reps, ops / best * 1e-9, ck, n_fb);
  return 0;
}
